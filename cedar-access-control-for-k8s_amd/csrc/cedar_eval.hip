// gfx950 evaluation kernel: tiered Cedar authorization for a batch of requests.
//
// Replaces, per request, the reference's
//   TieredPolicyStores.IsAuthorized (internal/server/store/store.go:25-42)
//     -> cedar-go (*PolicySet).IsAuthorized (call site store.go:31)
// Mapping onto CDNA4:
//   * one lane = one request; the 4 waves of a 256-thread block walk the tiers' policy stream in
//     lock step: each <=16 KiB chunk of policy records (descriptor + atoms + atom data) is copied
//     into LDS once per block with coalesced 16-byte loads, then every wave reads each record as a
//     wave-uniform LDS broadcast (4 x ds_read_b128 + v_readfirstlane), so all per-policy control
//     flow is scalar;
//   * scope tests are register-only: each request carries a 128-bit Bloom filter of its
//     principal / resource ancestor-or-self UIDs and a 64-bit mask over the image's action
//     table; the exact ancestor scan (independent, unrolled heap loads) runs only for lanes
//     whose Bloom bit is set; a `__ballot` skips the policy for the wave when no lane matches;
//   * "atomic" policies (when/unless = &&- or ||-chains of predicates over pre-resolved
//     attributes) run as 4-word atoms against an LDS table of pre-resolved (var, attribute)
//     values; other policies run as register bytecode (forward-only skip targets per lane);
//   * satisfied forbids/permits and errors are appended to per-request result lists; forbid
//     overrides permit; a tier falls through only on (Deny, no reasons, no errors).
// No MFMA: the work is integer compares, ID equality and short scans.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <algorithm>
#include <atomic>
#include <queue>
#include <vector>
#include <string>

#include "device.h"
#include "engine.h"
#include "image.h"

using namespace cgi;

namespace {

constexpr int BLOCK = 256;
// Diagnostic builds only (never the shipped library): CG_DBG removes one part of the pooled
// candidate pass to time the rest (results are wrong): 1 no atom evaluation, 2 no hit recording
// past the count, 3 no merge, 4 every lane loads the same head, 5 a set atom's element-hash match
// taken without the exact record compare (tools/gpu_session.sh dbg step).
#ifndef CG_DBG
#define CG_DBG 0
#endif

struct RV {
  uint32_t w0, w1, w2;
};

__device__ __forceinline__ uint32_t tag_of(const RV& v) { return v.w0 >> TAG_SHIFT; }

struct KArgs {
  const uint32_t* __restrict__ pstream;
  const uint32_t* __restrict__ chunks;
  const uint32_t* __restrict__ tier_cend;
  const uint32_t* __restrict__ cpool;
  const uint32_t* __restrict__ gstr_off;
  const uint8_t* __restrict__ gstr_bytes;
  const uint32_t* __restrict__ hot;
  const uint32_t* __restrict__ act;
  const uint32_t* __restrict__ heap;
  const uint32_t* __restrict__ req_idx;
  const uint32_t* __restrict__ bstr_off;
  const uint8_t* __restrict__ bstr_bytes;
  uint32_t* __restrict__ res;
  uint32_t* __restrict__ reasons_f;
  uint32_t* __restrict__ reasons_p;
  uint32_t* __restrict__ errs;
  const uint32_t* __restrict__ btab;     // scope index (indexed kernel)
  const uint32_t* __restrict__ bfilt;    // key filter (image.h filt_*)
  const uint32_t* __restrict__ bstream;
  const uint32_t* __restrict__ rows;     // columnar request rows (row_words each)
  uint32_t* __restrict__ lane;           // global lane area (GLANE stream kernel), lane_stride words per request
  const uint32_t* __restrict__ srows;    // static entities (image.h "static entities")
  const uint4* __restrict__ shash;
  unsigned long long* stats;             // probe-kernel work counters (STATS variant only)
  const uint32_t* n_dev;                 // follow-up pass: request count on the device (null: n_req)
  // first pass of a grouped batch: launch position -> request (the device sort's order, so that the
  // requests of a wave share scope-index buckets); results stay at the request's own index
  const uint32_t* ord;
  const uint32_t* __restrict__ grows;  // ... and its rows in that order (launch position k: grows + k * row_words)
  uint32_t n_pol, n_tiers, n_gstr, n_hot, n_act, amask_ok, n_req, capr, cape, bmask, fmask, row_words, combo_mask;
  uint32_t hlists;  // hot slots whose rows carry element-hash / prefix lists (image.h "set-membership
                    // keys"): the row's list-offset word of slot h is at its rank among them
  uint32_t l1filt;  // level-1 probes consult the key filter first (CEDARGPU_L1_FILTER=1: on, A/B)
  uint32_t l2filt;  // level-2 probes too, after the level-1 entry's own bloom (CEDARGPU_L2_FILTER)
  uint32_t slot_split;  // probes load a slot's first 16 B, the rest only on a key match (CEDARGPU_SLOT_SPLIT)
  uint32_t scan_lds;    // the scan stages key ancestors and hot values in LDS up front (CEDARGPU_SCAN_LDS)
  uint32_t scan_filt;   // the scan tests principal keys against the scope bitsets first (CEDARGPU_SCAN_FILT)
  const uint32_t* __restrict__ sctx;   // scope bitsets (image.h): context table, (bits, rank) rows,
  const uint32_t* __restrict__ sbits;  //   and every set bit's bucket at its rank
  const uint32_t* __restrict__ svals;
  const uint32_t* __restrict__ sbloom;  // context filter (image.h ctx_bloom_*; null: none)
  uint32_t sctx_mask, sbits_words;     // sbits_words 0: the image has none
  uint32_t n_kent;                     // key entities: a request's key-entity indices are below it
  uint32_t* bad_kidx;                  // count of requests whose indices are not (null: not counted)
  uint32_t l2_vmask, l2_lmask;         // hot slots with level-2 value / list keys (entity-principal combos)
  uint32_t scan_big;    // more scanned buckets than this: straight to the large stage (CEDARGPU_SCAN_BIG)
  uint32_t scan_heavy;  // more candidate heads than this: straight to the large stage (CEDARGPU_SCAN_HEAVY)
  uint32_t cnt_rank;    // merges of <= this many hits per request rank by counting (CEDARGPU_CNT_RANK)
  uint32_t n_static, smask, lane_stride;
  // split first pass (cedar_scan_kernel -> cedar_probe_kernel<.., SPLIT>), by position p of the
  // launch order (wave w = p / 8 holds positions 8w .. 8w + 7): p's bucket count at scan[p]
  // (SCAN_OVF: some of its buckets did not fit its wave's list); wave w's list total at scan_tot[w]
  // and its list at scan_list + w * 2 * WAVE_CAP: the wave's (first head | p % 8 << SCAN_SEG_SHIFT,
  // count | combo << SCAN_COMBO_SHIFT) pairs, packed in the order the scan found them
  uint32_t* scan;
  uint32_t* scan_tot;
  uint32_t* scan_list;
  uint32_t scan_n;
  // one-launch small batches (DevBatch::small): a request whose deciding list outgrows capr takes
  // an overflow slot (ovf_cnt: slots taken) and writes its whole result there, laid out like a
  // follow-up worklist entry (ids, res, reasons, errors) that cg_batch_wait folds in
  uint32_t* ovf_cnt;
  uint32_t *ovf_ids, *ovf_res, *ovf_rf, *ovf_er;
  uint32_t ovf_cap, ovf_capr, ovf_cape;
  // inline like atoms (image.h AK_LIKEI): like slots, their words' row offset, and the hot-row index
  // the probe kernel stages them at (0xFFFFFFFF: not staged; the atom reads the string's bytes)
  uint32_t lslot, like_off, like_base;
  // first pass of a grouped batch: runs of xcd_chunk consecutive waves (of the grouped order) on
  // one XCD (blocks are dealt round-robin over the 8 XCDs), so neighbours share that XCD's L2;
  // 0: block order (xcd_block)
  uint32_t xcd_chunk;
  uint32_t park;  // compact candidate pass: head atoms parked in LDS with the descriptor (2 or 4)
  uint32_t cls;   // candidate pass: a duplicate class's hit takes one slot, reported as RS_CLASS
};
// Block b of nb one-wave blocks -> the wave it runs: block b lands on XCD b % 8 as its (b / 8)-th
// block; chunks of C consecutive waves go to one XCD, chunks dealt round-robin (a bijection on the
// first multiple of 8C blocks, the rest in place). Speed only: any mapping is correct.
__device__ __forceinline__ uint32_t xcd_block(uint32_t b, uint32_t nb, uint32_t C) {
  if (!C) return b;
  const uint32_t full = nb - nb % (8u * C);
  if (b >= full) return b;
  const uint32_t x = b & 7u, j = b >> 3;
  return ((j / C) * 8u + x) * C + (j % C);
}
// SCAN_CAP: bucket pairs per request of a wave's list (WAVE_CAP per wave of 8 requests, packed:
// a request whose buckets do not all fit gets SCAN_OVF, and the large stage probes the index
// itself); a request with more than KArgs::scan_big buckets skips the candidate pass and goes to
// the large stage, which reads the list when it holds them all
// a follow-up worklist entry the first pass already finished (its id | FU_DONE): the follow-up
// launch skips it, the host folds its result as any other
constexpr uint32_t FU_DONE = 0x80000000u;
constexpr uint32_t SCAN_CAP = 96, SCAN_OVF = 0xFFFFFFFFu, SCAN_COUNT = (1u << 27) - 1, SCAN_COMBO_SHIFT = 27;
constexpr uint32_t WAVE_CAP = 8 * SCAN_CAP, SCAN_SEG_SHIFT = 27;  // (first heads stay below 2^27: EF_FIRST)
static_assert(WAVE_CAP >= 128, "the candidate pass reads two pairs per lane (128) before it knows the total");
// scan[i] | SCAN_HEAVY: the request's buckets hold more than a.scan_heavy candidate heads, so it
// goes straight to the large stage (the candidate pass would overflow its 64 hits and be redone)
constexpr uint32_t SCAN_HEAVY = 0x40000000u;

// Per-lane evaluation context. Every function taking it is force-inlined so that it stays in
// registers; the only non-inlined function (structural equality) takes plain pointers.
struct Ctx {
  const uint32_t* blk;    // request block (global)
  const uint32_t* cpool;  // image constant pool (global)
  uint32_t* lh;           // lane scratch (private): runtime-built sets/records
  const uint32_t* hot;
  const uint32_t* gstr_off;
  const uint8_t* gstr_bytes;
  const uint32_t* bstr_off;
  const uint8_t* bstr_bytes;
  uint32_t n_gstr;
  uint2* hotl;       // LDS hot table: hotl[h * hstride]
  uint32_t hstride;  // BLOCK (per-lane columns, request-per-lane kernel) or 1 (request-per-wave)
  uint32_t pt, pi, at, ai, rt, ri;
  uint32_t pidx, aidx, ridx;
  uint32_t nent;
  uint32_t p_anc, p_nanc, r_anc, r_nanc;  // offsets of ancestor pair arrays (in p_base / r_base), counts
  const uint32_t* p_base;                 // the request block, or the constant pool for a static entity
  const uint32_t* r_base;
  uint32_t a_anc, a_nanc;                 // action ancestors (probe kernel; stream kernel uses aidx)
  const uint32_t* srows;                  // static entities: rows and UID hash (n_static == 0: none)
  const uint4* shash;
  uint32_t n_static, smask;
  // first 8 principal ancestors, for the exact `in` test in registers (named scalars: an array
  // here would keep the whole context out of registers)
  uint32_t t0, i0, t1, i1, t2, i2, t3, i3, t4, i4, t5, i5, t6, i6, t7, i7;
  uint32_t pb0, pb1, pb2, pb3;            // principal ancestor-or-self Bloom
  uint32_t rb0, rb1, rb2, rb3;            // resource ancestor-or-self Bloom
  const uint32_t* rowx;                   // the row's element-hash list offsets (one per list slot), or null
  uint32_t lmask;                         // the list slots (KArgs::hlists)
  __device__ uint32_t hlist(uint32_t h) const {
    return (rowx && ((lmask >> h) & 1u)) ? rowx[__popc(lmask & ((1u << h) - 1u))] : 0xFFFFFFFFu;
  }
  static constexpr uint32_t lkb = 0xFFFFFFFFu;  // like words not staged (AK_LIKEI reads the bytes)
  static constexpr uint32_t lslot = 0u;
};

// Makes a value opaque to the optimizer. Used on context fields that feed a select: otherwise
// InstCombine turns `h == 0 ? c.pt : c.rt` into a load through a dynamic offset into the
// context, which forces the whole per-lane context into scratch memory.
__device__ __forceinline__ uint32_t opq(uint32_t x) {
  asm volatile("" : "+v"(x));
  return x;
}
// Selects among three per-lane values by a wave-uniform index (0, 1, else 2).
__device__ __forceinline__ uint32_t pick3(uint32_t h, uint32_t a, uint32_t b, uint32_t c) {
  return h == 0 ? opq(a) : (h == 1 ? opq(b) : opq(c));
}

// Value reference read (heap / constant pool / lane scratch).
__device__ __forceinline__ uint32_t rd3(const uint32_t* blk, const uint32_t* cpool, const uint32_t* lh, uint32_t ref,
                                        uint32_t i) {
  const uint32_t sp = ref >> SPACE_SHIFT, off = (ref & OFF_MASK) + i;
  if (sp == SP_HEAP) return blk[off];
  if (sp == SP_CPOOL) return cpool[off];
  return lh[off];
}
template <class CT>
__device__ __forceinline__ uint32_t rd(const CT& c, uint32_t ref, uint32_t i) { return rd3(c.blk, c.cpool, c.lh, ref, i); }

__device__ __forceinline__ RV load_val3(const uint32_t* blk, const uint32_t* cpool, const uint32_t* lh, uint32_t w0,
                                        uint32_t w1) {
  const uint32_t t = w0 >> TAG_SHIFT;
  if (t == T_LONG) return RV{mk_w0(T_LONG, 0), w1, ((int32_t)w1 < 0) ? 0xFFFFFFFFu : 0u};
  if (t == T_LONGREF) {
    const uint32_t ref = w0 & X_MASK;
    return RV{mk_w0(T_LONG, 0), rd3(blk, cpool, lh, ref, 0), rd3(blk, cpool, lh, ref, 1)};
  }
  return RV{w0, w1, 0};
}
template <class CT>
__device__ __forceinline__ RV load_val(const CT& c, uint32_t w0, uint32_t w1) { return load_val3(c.blk, c.cpool, c.lh, w0, w1); }

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

// ---- equality -------------------------------------------------------------------------------
// Shallow comparison: decides everything except (set, set) and (record, record) pairs.
// Returns 0 false, 1 true, 2 = needs a structural comparison.
__device__ __forceinline__ uint32_t veq_shallow(const uint32_t* blk, const uint32_t* cpool, const uint32_t* lh,
                                                const RV& a, const RV& b) {
  const uint32_t ta = tag_of(a), tb = tag_of(b);
  if (ta != tb) return 0u;
  switch (ta) {
    case T_BOOL:
    case T_STR: return a.w1 == b.w1 ? 1u : 0u;
    case T_LONG: return (a.w1 == b.w1 && a.w2 == b.w2) ? 1u : 0u;
    case T_ENT: return (a.w0 == b.w0 && a.w1 == b.w1) ? 1u : 0u;
    case T_DEC: {
      const uint32_t ra = a.w0 & X_MASK, rb = b.w0 & X_MASK;
      return (rd3(blk, cpool, lh, ra, 0) == rd3(blk, cpool, lh, rb, 0) && rd3(blk, cpool, lh, ra, 1) == rd3(blk, cpool, lh, rb, 1)) ? 1u : 0u;
    }
    case T_IP: {
      const uint32_t ra = a.w0 & X_MASK, rb = b.w0 & X_MASK;
      for (uint32_t k = 0; k < 5; k++) if (rd3(blk, cpool, lh, ra, k) != rd3(blk, cpool, lh, rb, k)) return 0u;
      return 1u;
    }
    case T_SET:
    case T_REC: return (ta == T_REC && a.w1 != b.w1) ? 0u : 2u;  // records: unique keys, counts must agree
    default: return 0u;
  }
}

// Structural equality of two sets or two records, iterative over an explicit frame stack (no
// recursion): set equality is mutual inclusion (lane-built sets may hold duplicates), record
// equality is equal sorted key lists with equal values. Returns 0 false, 1 true, 2 nesting
// beyond VAL_DEPTH (reported as E_DEPTH).
__device__ __noinline__ uint32_t veq_struct(const uint32_t* blk, const uint32_t* cpool, const uint32_t* lh, RV a, RV b) {
  struct Frame {
    uint32_t ra, rb, na, nb;
    uint32_t set, phase, i, j;  // set: 1 set, 0 record; phase: 0 a-in-b, 1 b-in-a
  };
  Frame st[VAL_DEPTH];
  uint32_t sp = 0;
  st[sp++] = Frame{a.w0 & X_MASK, b.w0 & X_MASK, a.w1, b.w1, tag_of(a) == T_SET ? 1u : 0u, 0, 0, 0};
  bool have = false, ret = false;  // result of the child frame just popped
  while (sp > 0) {
    Frame& f = st[sp - 1];
    bool done = false, res = false, pushed = false;
    if (f.set) {
      if (have) {  // child compared outer[i] with inner[j]
        have = false;
        if (ret) { f.i++; f.j = 0; } else { f.j++; }
      }
      for (;;) {
        const uint32_t no = f.phase ? f.nb : f.na, ni = f.phase ? f.na : f.nb;
        if (f.i >= no) {
          if (f.phase == 0) { f.phase = 1; f.i = 0; f.j = 0; continue; }
          done = true; res = true;
          break;
        }
        if (f.j >= ni) { done = true; res = false; break; }
        const uint32_t ro = f.phase ? f.rb : f.ra, rn = f.phase ? f.ra : f.rb;
        const RV x = load_val3(blk, cpool, lh, rd3(blk, cpool, lh, ro, 1 + 2 * f.i), rd3(blk, cpool, lh, ro, 2 + 2 * f.i));
        const RV y = load_val3(blk, cpool, lh, rd3(blk, cpool, lh, rn, 1 + 2 * f.j), rd3(blk, cpool, lh, rn, 2 + 2 * f.j));
        const uint32_t s = veq_shallow(blk, cpool, lh, x, y);
        if (s == 2u) {
          if (sp >= VAL_DEPTH) return 2u;
          st[sp++] = Frame{x.w0 & X_MASK, y.w0 & X_MASK, x.w1, y.w1, tag_of(x) == T_SET ? 1u : 0u, 0, 0, 0};
          pushed = true;
          break;
        }
        if (s) { f.i++; f.j = 0; } else { f.j++; }
      }
    } else {
      if (have) {
        have = false;
        if (!ret) { done = true; res = false; } else { f.i++; }
      }
      while (!done) {
        if (f.i >= f.na) { done = true; res = true; break; }
        if (rd3(blk, cpool, lh, f.ra, 1 + 3 * f.i) != rd3(blk, cpool, lh, f.rb, 1 + 3 * f.i)) { done = true; res = false; break; }
        const RV x = load_val3(blk, cpool, lh, rd3(blk, cpool, lh, f.ra, 2 + 3 * f.i), rd3(blk, cpool, lh, f.ra, 3 + 3 * f.i));
        const RV y = load_val3(blk, cpool, lh, rd3(blk, cpool, lh, f.rb, 2 + 3 * f.i), rd3(blk, cpool, lh, f.rb, 3 + 3 * f.i));
        const uint32_t s = veq_shallow(blk, cpool, lh, x, y);
        if (s == 2u) {
          if (sp >= VAL_DEPTH) return 2u;
          st[sp++] = Frame{x.w0 & X_MASK, y.w0 & X_MASK, x.w1, y.w1, tag_of(x) == T_SET ? 1u : 0u, 0, 0, 0};
          pushed = true;
          break;
        }
        if (!s) { done = true; res = false; break; }
        f.i++;
      }
    }
    if (pushed) continue;
    if (done) {
      sp--;
      have = true;
      ret = res;
    }
  }
  return ret ? 1u : 0u;
}

// full equality; `deep` set when nesting exceeds the device limit, or (STRUCT = false, the probe
// kernel) whenever a set/record comparison is needed: the request then re-runs on the stream kernel
template <bool STRUCT = true, class CT>
__device__ __forceinline__ bool veq(const CT& c, const RV& a, const RV& b, bool& deep) {
  const uint32_t s = veq_shallow(c.blk, c.cpool, c.lh, a, b);
  if (s != 2u) return s == 1u;
  if (!STRUCT) { deep = true; return false; }
  const uint32_t r = veq_struct(c.blk, c.cpool, c.lh, a, b);
  if (r == 2u) deep = true;
  return r == 1u;
}

// primitive equality against a register-form constant (tags equal and payload equal)
__device__ __forceinline__ bool prim_eq(const RV& v, uint32_t c0, uint32_t c1, uint32_t c2) {
  if (v.w0 >> TAG_SHIFT != c0 >> TAG_SHIFT) return false;
  switch (c0 >> TAG_SHIFT) {
    case T_LONG: return v.w1 == c1 && v.w2 == c2;
    case T_ENT: return v.w0 == c0 && v.w1 == c1;
    default: return v.w1 == c1;
  }
}

// ---- records / entities (request data is always in the heap) -------------------------------
__device__ __forceinline__ bool rec_get(const Ctx& c, const RV& rec, uint32_t key, RV& out) {
  const uint32_t ref = rec.w0 & X_MASK, n = rec.w1;
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (rd(c, ref, 1 + 3 * mid) < key) lo = mid + 1;
    else hi = mid;
  }
  if (lo < n && rd(c, ref, 1 + 3 * lo) == key) {
    out = load_val(c, rd(c, ref, 2 + 3 * lo), rd(c, ref, 3 + 3 * lo));
    return true;
  }
  return false;
}
// heap record lookup, memory form (hot table fill)
__device__ __forceinline__ bool rec_get_heap(const uint32_t* blk, uint32_t rw0, uint32_t n, uint32_t key, uint2& out) {
  const uint32_t off = rw0 & OFF_MASK;
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (blk[off + 1 + 3 * mid] < key) lo = mid + 1;
    else hi = mid;
  }
  if (lo < n && blk[off + 1 + 3 * lo] == key) {
    out = make_uint2(blk[off + 2 + 3 * lo], blk[off + 3 + 3 * lo]);
    return true;
  }
  return false;
}

// A UID the request's table lacks may be one of the image's static entities (merged EntityMap).
__device__ __forceinline__ uint32_t static_find(const Ctx& c, uint32_t et, uint32_t ei) {
  if (!c.n_static) return NO_ENT;
  for (uint32_t h = uid_hash(et, ei) & c.smask;; h = (h + 1) & c.smask) {
    const uint4 sl = c.shash[h];
    if (sl.z == 0) return NO_ENT;
    if (sl.x == et && sl.y == ei) return ENT_STATIC | (sl.z - 1);
  }
}

__device__ __forceinline__ uint32_t find_ent(const Ctx& c, uint32_t et, uint32_t ei) {
  if (et == c.pt && ei == c.pi) return opq(c.pidx);
  if (et == c.rt && ei == c.ri) return opq(c.ridx);
  if (et == c.at && ei == c.ai) return opq(c.aidx);
  for (uint32_t i = 0; i < c.nent; i++) {
    const uint32_t* row = c.blk + RH_WORDS + i * ENT_WORDS;
    if (row[ER_TYPE] == et && row[ER_ID] == ei) return i;
  }
  return static_find(c, et, ei);
}

// entity row of a table index or a static index
__device__ __forceinline__ const uint32_t* ent_row(const Ctx& c, uint32_t idx) {
  return (idx & ENT_STATIC) ? c.srows + (size_t)(idx & ~ENT_STATIC) * ENT_WORDS : c.blk + RH_WORDS + idx * ENT_WORDS;
}

// exact membership in an ancestor list: pairs at blk[off + 2k] (off signed: a request's lists sit
// ahead of its block, image.h "ancestor lists"), independent loads, 4 per step
__device__ __forceinline__ bool anc_scan(const uint32_t* blk, uint32_t off, uint32_t n, uint32_t qt, uint32_t qi) {
  const uint32_t* l = blk + (int32_t)off;
  bool f = false;
  uint32_t k = 0;
  for (; k + 4 <= n && !f; k += 4) {
    const uint32_t* q = l + 2 * k;
    const uint32_t t0 = q[0], i0 = q[1], t1 = q[2], i1 = q[3], t2 = q[4], i2 = q[5], t3 = q[6], i3 = q[7];
    f = (t0 == qt && i0 == qi) | (t1 == qt && i1 == qi) | (t2 == qt && i2 == qi) | (t3 == qt && i3 == qi);
  }
  for (; k < n && !f; k++) f = l[2 * k] == qt && l[2 * k + 1] == qi;
  return f;
}

// ancestor list of an entity: pairs at base[off + 2k] (a static entity's closure row lives in the
// constant pool; a table entity's list in the heap, at a signed block-relative ref)
__device__ __forceinline__ void anc_of(const Ctx& c, uint32_t idx, const uint32_t*& base, uint32_t& off, uint32_t& n) {
  base = c.blk; off = 0; n = 0;
  if (idx == NO_ENT) return;
  const uint32_t ref = ent_row(c, idx)[ER_ANC] & OFF_MASK;
  const uint32_t* l = (idx & ENT_STATIC) ? c.cpool + ref : c.blk + sext26(ref);
  n = l[0];
  base = l + 1;
}

__device__ __forceinline__ bool anc_has(const Ctx& c, uint32_t idx, uint32_t qt, uint32_t qi) {
  const uint32_t* base;
  uint32_t off, n;
  anc_of(c, idx, base, off, n);
  return anc_scan(base, off, n, qt, qi);
}

__device__ __forceinline__ bool ent_in(const Ctx& c, uint32_t et, uint32_t ei, uint32_t qt, uint32_t qi) {
  if (et == qt && ei == qi) return true;
  return anc_has(c, find_ent(c, et, ei), qt, qi);
}

__device__ __forceinline__ bool bloom_test(uint32_t b0, uint32_t b1, uint32_t b2, uint32_t b3, uint32_t bit) {
  const uint32_t w = bit < 64 ? (bit < 32 ? b0 : b1) : (bit < 96 ? b2 : b3);
  return (w >> (bit & 31)) & 1u;
}
__device__ __forceinline__ void bloom_add(uint32_t& b0, uint32_t& b1, uint32_t& b2, uint32_t& b3, uint32_t bit) {
  const uint32_t m = 1u << (bit & 31);
  b0 |= bit < 32 ? m : 0u;
  b1 |= (bit >= 32 && bit < 64) ? m : 0u;
  b2 |= (bit >= 64 && bit < 96) ? m : 0u;
  b3 |= bit >= 96 ? m : 0u;
}

// principal / resource `in E` with the Bloom shortcut (bit = uid_bloom_bit(et, ei), uniform)
__device__ __forceinline__ bool p_in(const Ctx& c, uint32_t et, uint32_t ei, uint32_t bit) {
  if (c.pt == et && c.pi == ei) return true;
  if (!bloom_test(c.pb0, c.pb1, c.pb2, c.pb3, bit)) return false;
  // unused entries hold ~0u
  bool f = ((c.t0 == et) & (c.i0 == ei)) | ((c.t1 == et) & (c.i1 == ei)) | ((c.t2 == et) & (c.i2 == ei)) |
           ((c.t3 == et) & (c.i3 == ei)) | ((c.t4 == et) & (c.i4 == ei)) | ((c.t5 == et) & (c.i5 == ei)) |
           ((c.t6 == et) & (c.i6 == ei)) | ((c.t7 == et) & (c.i7 == ei));
  if (!f && c.p_nanc > 8) f = anc_scan(c.p_base, c.p_anc + 16, c.p_nanc - 8, et, ei);
  return f;
}
__device__ __forceinline__ bool r_in(const Ctx& c, uint32_t et, uint32_t ei, uint32_t bit) {
  if (c.rt == et && c.ri == ei) return true;
  if (!bloom_test(c.rb0, c.rb1, c.rb2, c.rb3, bit)) return false;
  return anc_scan(c.r_base, c.r_anc, c.r_nanc, et, ei);
}

// ---- strings / like -------------------------------------------------------------------------
template <class CT>
__device__ __forceinline__ void str_span(const CT& c, uint32_t sid, const uint8_t*& p, uint32_t& len) {
  if (sid < c.n_gstr) {
    const uint32_t o = c.gstr_off[sid];
    len = c.gstr_off[sid + 1] - o;
    p = c.gstr_bytes + o;
  } else {
    const uint32_t j = c.blk[RH_SBASE] + (sid - c.n_gstr);  // request-local id -> batch string
    const uint32_t o = c.bstr_off[j];
    len = c.bstr_off[j + 1] - o;
    p = c.bstr_bytes + o;
  }
}

// pattern literal bytes: 4 per word, little-endian
__device__ __forceinline__ uint32_t pat_byte(const uint32_t* w, uint32_t k) { return (w[k >> 2] >> (8 * (k & 3))) & 0xFFu; }

__device__ __forceinline__ bool lit_at(const uint8_t* s, uint32_t pos, const uint32_t* w, uint32_t n) {
  bool ok = true;
  uint32_t k = 0;
  for (; k + 4 <= n && ok; k += 4) {  // 4 independent byte loads per step
    const uint32_t x = (uint32_t)s[pos + k] | ((uint32_t)s[pos + k + 1] << 8) | ((uint32_t)s[pos + k + 2] << 16) |
                       ((uint32_t)s[pos + k + 3] << 24);
    ok = x == w[k >> 2];
  }
  for (; k < n && ok; k++) ok = s[pos + k] == pat_byte(w, k);
  return ok;
}

// s[pos, pos + n) equals the literal packed in w (4 bytes per word): LIT_U bytes a round, their
// loads issued together (a byte loop that stops at the first mismatch makes every byte load wait
// for the previous compare: a `like "prod-*"` prefix was 5 dependent trips to memory)
constexpr uint32_t LIT_U = 8;
template <class P>
__device__ __forceinline__ bool lit_eq(const uint8_t* s, uint32_t pos, P w, uint32_t n) {
  for (uint32_t k0 = 0; k0 < n; k0 += LIT_U) {
    uint32_t b[LIT_U];
#pragma unroll
    for (uint32_t j = 0; j < LIT_U; j++) b[j] = k0 + j < n ? (uint32_t)s[pos + k0 + j] : 0u;
    bool ok = true;
#pragma unroll
    for (uint32_t j = 0; j < LIT_U; j++)
      if (k0 + j < n) ok = ok && b[j] == ((w[(k0 + j) >> 2] >> (8 * ((k0 + j) & 3))) & 0xFFu);
    if (!ok) return false;
  }
  return true;
}

// `pw` points at a compiled pattern (LDS record data or global constant pool)
template <class CT, class P>
__device__ __forceinline__ bool like_match(const CT& c, uint32_t sid, P pw) {
  const uint8_t* s;
  uint32_t slen;
  str_span(c, sid, s, slen);
  const uint32_t flags = pw[0];
  uint32_t q = 1;
  const uint32_t plen = pw[q];
  const uint32_t pq = q + 1;
  q += 1 + ((plen + 3) >> 2);
  if (!(flags & 1)) {
    if (slen != plen) return false;
    return lit_eq(s, 0u, pw + pq, plen);
  }
  const uint32_t sl = pw[q];
  const uint32_t sq = q + 1;
  q += 1 + ((sl + 3) >> 2);
  if (slen < plen + sl) return false;
  if (!lit_eq(s, 0u, pw + pq, plen) || !lit_eq(s, slen - sl, pw + sq, sl)) return false;
  uint32_t pos = plen;
  const uint32_t end = slen - sl;
  const uint32_t nmid = flags >> 8;
  for (uint32_t m = 0; m < nmid; m++) {
    const uint32_t ml = pw[q];
    const uint32_t mq = q + 1;
    q += 1 + ((ml + 3) >> 2);
    bool found = false;
    while (pos + ml <= end && !found) {
      bool eq = true;
      for (uint32_t k = 0; k < ml && eq; k++) eq = s[pos + k] == ((pw[mq + (k >> 2)] >> (8 * (k & 3))) & 0xFFu);
      if (eq) found = true;
      else pos++;
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

// Hot slot h of this lane: the value (memory form) or a status word (tag NONE; x = error code |
// HS_FINAL; y = block offset of the error detail the encoder resolved, image.h "hot paths").
template <class CT>
__device__ __forceinline__ uint2 hot_get(const CT& c, uint32_t h) { return c.hotl[h * c.hstride]; }
__device__ __forceinline__ bool hot_ok(uint2 v) { return (v.x >> TAG_SHIFT) != T_NONE; }
// `has` on a hot path: present -> 1, absent at the final step -> 0, failing earlier -> 2 (error)
__device__ __forceinline__ uint32_t hot_has(uint2 v) { return hot_ok(v) ? 1u : ((v.x & HS_FINAL) ? 0u : 2u); }
// The error attribute access raises for a non-present hot slot.
template <class CT>
__device__ __forceinline__ void hot_err(const CT& c, uint32_t h, uint2 v, Err& e) {
  const uint32_t* d = c.blk + v.y;
  const uint32_t w = d[0];
  e.code = w & 0xFF;
  e.aux = w >> 8;
  e.k = d[1];
  e.et = d[2];
  e.ei = d[3];
}

// AK_LIKEI: string sid (the value of hot slot h) like the inline pattern (p0, p1: prefix then suffix
// bytes; f: prefix length | suffix length << 4 | star << 8). The string's length and first / last 8
// bytes come from the staged like words (c.lkb), else from the string itself.
template <class CT>
__device__ __forceinline__ bool likei(const CT& c, uint32_t h, uint32_t sid, uint32_t p0, uint32_t p1, uint32_t f) {
  uint32_t len;
  uint64_t pre = 0, suf = 0;
  // (only a slot of c.lslot has staged words: an atom lowered without them, e.g. one an incremental
  // build kept from an image compiled with another like-words choice, reads the string)
  if (c.lkb != 0xFFFFFFFFu && h < 32u && ((c.lslot >> h) & 1u)) {
    const uint32_t k = c.lkb + 3u * (uint32_t)__popc(c.lslot & ((1u << h) - 1u));
    const uint2 x = hot_get(c, k), y = hot_get(c, k + 1), z = hot_get(c, k + 2);
    len = x.x;
    pre = ((uint64_t)y.x << 32) | x.y;
    suf = ((uint64_t)z.x << 32) | y.y;
  } else {
    const uint8_t* s;
    str_span(c, sid, s, len);
    const uint32_t n = min(len, 8u);
#pragma unroll
    for (uint32_t j = 0; j < 8; j++)
      if (j < n) {
        pre |= (uint64_t)s[j] << (8 * j);
        suf |= (uint64_t)s[len - 1 - j] << (8 * (7 - j));
      }
  }
  const uint32_t pl = f & 15u, sl = (f >> 4) & 15u;
  const uint64_t pat = ((uint64_t)p1 << 32) | p0;
  auto msk = [](uint32_t n) { return n >= 8 ? ~0ull : ((1ull << (8 * n)) - 1ull); };
  if (!(f & 256u)) return len == pl && ((pre ^ pat) & msk(pl)) == 0;
  if (len < pl + sl || ((pre ^ pat) & msk(pl)) != 0) return false;
  if (!sl) return true;
  return (suf >> (64 - 8 * sl)) == ((pat >> (8 * pl)) & msk(sl));  // (sl >= 1: pl <= 7)
}

// ---- atoms ---------------------------------------------------------------------------------
// rec = this policy's LDS record (atom data lives there). Returns 0 false, 1 true, 2 error.
// AK_RECSET helpers: compare a request value with one template operand (const or hot hole).
template <bool STRUCT, class CT>
__device__ __forceinline__ bool rs_opnd_eq(const CT& c, const RV& x, uint32_t kind, uint32_t a, uint32_t b, uint32_t d,
                                           bool& deep) {
  if (kind == RF_CONST) return prim_eq(x, a, b, d);
  const uint2 hv = hot_get(c, a);  // holes were checked present before matching
  return veq<STRUCT>(c, x, load_val(c, hv.x, hv.y), deep);
}
// set-literal field: x (must be a set) equals the literal list by mutual inclusion
template <bool STRUCT, class CT>
__device__ __forceinline__ bool rs_set_eq(const CT& c, const RV& x, const uint32_t* el, uint32_t n, bool& deep) {
  if (tag_of(x) != T_SET) return false;
  const uint32_t ref = x.w0 & X_MASK, m = x.w1;
  for (uint32_t i = 0; i < m; i++) {
    const RV xi = load_val(c, rd(c, ref, 1 + 2 * i), rd(c, ref, 2 + 2 * i));
    bool f = false;
    for (uint32_t j = 0; j < n && !f; j++) f = rs_opnd_eq<STRUCT>(c, xi, el[4 * j], el[4 * j + 1], el[4 * j + 2], el[4 * j + 3], deep);
    if (!f) return false;
  }
  for (uint32_t j = 0; j < n; j++) {
    bool f = false;
    for (uint32_t i = 0; i < m && !f; i++) {
      const RV xi = load_val(c, rd(c, ref, 1 + 2 * i), rd(c, ref, 2 + 2 * i));
      f = rs_opnd_eq<STRUCT>(c, xi, el[4 * j], el[4 * j + 1], el[4 * j + 2], el[4 * j + 3], deep);
    }
    if (!f) return false;
  }
  return true;
}
// record x == template t (sorted keys, exact key set)
template <bool STRUCT, class CT>
__device__ __forceinline__ bool rs_rec_eq(const CT& c, const uint32_t* rec, const RV& x, const uint32_t* t, bool& deep) {
  const uint32_t nk = t[0];
  if (tag_of(x) != T_REC || x.w1 != nk) return false;
  const uint32_t ref = x.w0 & X_MASK;
  for (uint32_t k = 0; k < nk; k++) {
    const uint32_t* f = t + 1 + RS_FIELD_WORDS * k;
    if (rd(c, ref, 1 + 3 * k) != f[0]) return false;
    const RV xf = load_val(c, rd(c, ref, 2 + 3 * k), rd(c, ref, 3 + 3 * k));
    const bool q = f[1] == RF_SETLIT ? rs_set_eq<STRUCT>(c, xf, rec + f[2], f[3], deep)
                                     : rs_opnd_eq<STRUCT>(c, xf, f[1], f[2], f[3], f[4], deep);
    if (!q) return false;
  }
  return true;
}

// var h (0 principal, 1 action, 2 resource) `in` entity (qt, qi); bit = its Bloom bit
__device__ __forceinline__ bool var_in(const Ctx& c, uint32_t h, uint32_t qt, uint32_t qi, uint32_t bit) {
  if (h == 0) return p_in(c, qt, qi, bit);
  if (h == 2) return r_in(c, qt, qi, bit);
  if (c.aidx == NO_ENT && c.a_nanc) return (c.at == qt && c.ai == qi) || anc_scan(c.blk, c.a_anc, c.a_nanc, qt, qi);
  return (c.at == qt && c.ai == qi) || anc_has(c, c.aidx, qt, qi);
}

template <bool STRUCT, class CT>
__device__ __forceinline__ uint32_t eval_atom(const CT& c, const uint32_t* rec, uint32_t kind, uint32_t h, uint32_t w1,
                                              uint32_t w2, uint32_t w3, Err& e) {
  if (kind == AK_IS) {
    return pick3(h, c.pt, c.at, c.rt) == w1 ? 1u : 0u;
  }
  if (kind == AK_IN) return var_in(c, h, w1, w2, w3) ? 1u : 0u;
  if (kind == AK_TRUE) return 1u;
  if (kind == AK_EQV) return (pick3(h, c.pt, c.at, c.rt) == w1 && pick3(h, c.pi, c.ai, c.ri) == w2) ? 1u : 0u;
  if (kind == AK_INANY) {
    bool f = false;
    for (uint32_t k = 0; k < w2 && !f; k++) {
      const uint32_t qt = rec[w1 + 2 * k], qi = rec[w1 + 2 * k + 1];
      f = var_in(c, h, qt, qi, uid_bloom_bit(qt, qi));
    }
    return f ? 1u : 0u;
  }
  const uint2 hv = hot_get(c, h);
  if (kind == AK_HAS) {
    const uint32_t q = hot_has(hv);
    if (q == 2u) hot_err(c, h, hv, e);
    return q;
  }
  if (!hot_ok(hv)) { hot_err(c, h, hv, e); return 2u; }
  const RV v = load_val(c, hv.x, hv.y);
  switch (kind) {
    case AK_BOOL:
      if (tag_of(v) != T_BOOL) { type_err(e, TN_BOOL, v); return 2u; }
      return v.w1;
    case AK_EQ: return prim_eq(v, w1, w2, w3) ? 1u : 0u;
    case AK_EQH: {
      const uint2 hv2 = hot_get(c, w1);
      if (!hot_ok(hv2)) { hot_err(c, w1, hv2, e); return 2u; }
      bool deep = false;
      const bool q = veq<STRUCT>(c, v, load_val(c, hv2.x, hv2.y), deep);
      if (deep) { if (!STRUCT) return 3u; e.code = E_DEPTH; return 2u; }
      return q ? 1u : 0u;
    }
    case AK_INSET: {
      bool f = false;
      for (uint32_t k = 0; k < w2 && !f; k++) {
        const uint32_t* el = rec + w1 + 3 * k;
        f = prim_eq(v, el[0], el[1], el[2]);  // per-lane policy in the index kernel: no readfirstlane
      }
      return f ? 1u : 0u;
    }
    case AK_CONTAINS: {
      if (tag_of(v) != T_SET) { type_err(e, TN_SET, v); return 2u; }
      const uint32_t ref = v.w0 & X_MASK, n = v.w1;
      const uint32_t hl = c.hlist(h);
      uint32_t th;
      if (hl != 0xFFFFFFFFu && reg_chash(w1, w2, w3, th)) {  // element hashes first, values on a match
        bool f = false;
        for (uint32_t k = 0; k < n && !f; k++)
          if (c.blk[hl + 1 + k] == th) f = prim_eq(load_val(c, rd(c, ref, 1 + 2 * k), rd(c, ref, 2 + 2 * k)), w1, w2, w3);
        return f ? 1u : 0u;
      }
      bool f = false;
      for (uint32_t k = 0; k < n && !f; k++) f = prim_eq(load_val(c, rd(c, ref, 1 + 2 * k), rd(c, ref, 2 + 2 * k)), w1, w2, w3);
      return f ? 1u : 0u;
    }
    case AK_LIKE:
      if (tag_of(v) != T_STR) { type_err(e, TN_STRING, v); return 2u; }
      return like_match(c, v.w1, rec + w1) ? 1u : 0u;
    case AK_LIKEI:
      if (tag_of(v) != T_STR) { type_err(e, TN_STRING, v); return 2u; }
      return likei(c, h, v.w1, w1, w2, w3) ? 1u : 0u;
    case AK_INSTR:
      return (tag_of(v) == T_STR && (v.w1 == w1 || v.w1 == w2 || v.w1 == w3)) ? 1u : 0u;
    case AK_RECSET: {
      const uint32_t* d = rec + w1;
      const uint32_t nh = d[0];
      for (uint32_t k = 0; k < nh; k++) {  // argument evaluation precedes the receiver type check
        const uint2 hv2 = hot_get(c, d[1 + k]);
        if (!hot_ok(hv2)) { hot_err(c, d[1 + k], hv2, e); return 2u; }
      }
      if (tag_of(v) != T_SET) { type_err(e, TN_SET, v); return 2u; }
      const uint32_t ref = v.w0 & X_MASK, n = v.w1;
      bool f = false, deep = false;
      const uint32_t hl = c.hlist(h);
      if (hl != 0xFFFFFFFFu) {  // templates of primitives (constants, primitive holes): hashes first
        bool hashable = true;
        const uint32_t* t = d + 1 + nh;
        for (uint32_t j = 0; j < w2 && !f && hashable; j++) {
          const uint32_t nk = t[0];
          uint32_t th = chash_mix(CHASH_REC, nk);
          for (uint32_t q = 0; q < nk && hashable; q++) {
            const uint32_t* fl = t + 1 + RS_FIELD_WORDS * q;
            uint32_t fh = 0;
            // (a field that is no primitive hashes by its tag alone, as the encoder hashes a record
            // element's nested sets and records (encode_impl.h mem_chash): equal records still hash
            // alike, and a hash match is compared exactly)
            if (fl[1] == RF_CONST) {
              hashable = reg_chash(fl[2], fl[3], fl[4], fh);
            } else if (fl[1] == RF_HOLE) {
              const uint2 hv3 = hot_get(c, fl[2]);
              const RV hx = load_val(c, hv3.x, hv3.y);
              if (!reg_chash(hx.w0, hx.w1, hx.w2, fh)) fh = chash_prim(tag_of(hx), 0u, 0u);
            } else {  // RF_SETLIT: a set
              fh = chash_prim(T_SET, 0u, 0u);
            }
            th = chash_mix(chash_mix(th, fl[0]), fh);
          }
          for (uint32_t i = 0; i < n && !f && hashable; i++)
            if (c.blk[hl + 1 + i] == th) f = CG_DBG == 5 ? true : rs_rec_eq<STRUCT>(c, rec, load_val(c, rd(c, ref, 1 + 2 * i), rd(c, ref, 2 + 2 * i)), t, deep);
          t += 1 + RS_FIELD_WORDS * nk;
        }
        if (hashable) {
          if (deep) { if (!STRUCT) return 3u; e.code = E_DEPTH; return 2u; }
          return f ? 1u : 0u;
        }
        f = deep = false;  // a template the hashes do not cover: the element-by-element path
      }
      for (uint32_t i = 0; i < n && !f; i++) {
        const RV x = load_val(c, rd(c, ref, 1 + 2 * i), rd(c, ref, 2 + 2 * i));
        if (tag_of(x) != T_REC) continue;
        const uint32_t* t = d + 1 + nh;
        for (uint32_t j = 0; j < w2 && !f; j++) {
          f = rs_rec_eq<STRUCT>(c, rec, x, t, deep);
          t += 1 + RS_FIELD_WORDS * t[0];
        }
      }
      if (deep) { if (!STRUCT) return 3u; e.code = E_DEPTH; return 2u; }
      return f ? 1u : 0u;
    }
    case AK_LCMP: {
      if (tag_of(v) != T_LONG) { type_err(e, TN_LONG, v); return 2u; }
      const int64_t x = as_i64(v), y = (int64_t)(((uint64_t)w3 << 32) | w2);
      const bool r = w1 == 0 ? x < y : w1 == 1 ? x <= y : w1 == 2 ? x > y : x >= y;
      return r ? 1u : 0u;
    }
    default: return 0u;
  }
}

// ---- bytecode (general policies) ---------------------------------------------------------
// Runs one policy program for the lanes with `run` set. On return run = satisfied, err = error.
// `code` points into the LDS-staged record.
// Register file of the bytecode machine: 24 local scalars a0..c7 (never address-taken, so
// they stay in VGPRs) selected by wave-uniform operands through macro-expanded switches; slots 8..
// (deep expressions) spill to the policy's lane scratch at sb (image.h MAX_SLOTS).
#define CG_SLOT_GET(i, out) \
  do { \
    switch (i) { \
      case 0: (out) = RV{a0, b0, c0}; break; \
      case 1: (out) = RV{a1, b1, c1}; break; \
      case 2: (out) = RV{a2, b2, c2}; break; \
      case 3: (out) = RV{a3, b3, c3}; break; \
      case 4: (out) = RV{a4, b4, c4}; break; \
      case 5: (out) = RV{a5, b5, c5}; break; \
      case 6: (out) = RV{a6, b6, c6}; break; \
      case 7: (out) = RV{a7, b7, c7}; break; \
      default: { const uint32_t* sp_ = c.lh + sb + 3 * ((i) - 8); (out) = RV{sp_[0], sp_[1], sp_[2]}; } break; \
    } \
  } while (0)
#define CG_SLOT_SET(i, v) \
  do { \
    switch (i) { \
      case 0: a0 = (v).w0; b0 = (v).w1; c0 = (v).w2; break; \
      case 1: a1 = (v).w0; b1 = (v).w1; c1 = (v).w2; break; \
      case 2: a2 = (v).w0; b2 = (v).w1; c2 = (v).w2; break; \
      case 3: a3 = (v).w0; b3 = (v).w1; c3 = (v).w2; break; \
      case 4: a4 = (v).w0; b4 = (v).w1; c4 = (v).w2; break; \
      case 5: a5 = (v).w0; b5 = (v).w1; c5 = (v).w2; break; \
      case 6: a6 = (v).w0; b6 = (v).w1; c6 = (v).w2; break; \
      case 7: a7 = (v).w0; b7 = (v).w1; c7 = (v).w2; break; \
      default: { uint32_t* sp_ = c.lh + sb + 3 * ((i) - 8); sp_[0] = (v).w0; sp_[1] = (v).w1; sp_[2] = (v).w2; } break; \
    } \
  } while (0)
static_assert(NSLOT == 8, "CG_SLOT_GET/SET enumerate 8 register slots");

// ip(s) / decimal(s) of a runtime string, as the host parser (parser.cpp parse_ip / parse_decimal)
__device__ __forceinline__ bool dev_digit(uint32_t ch) { return ch - '0' < 10u; }
__device__ __forceinline__ int dev_hex(uint32_t ch) {
  if (ch - '0' < 10u) return (int)(ch - '0');
  if (ch - 'a' < 6u) return (int)(ch - 'a' + 10);
  if (ch - 'A' < 6u) return (int)(ch - 'A' + 10);
  return -1;
}
__device__ bool dev_parse_decimal(const uint8_t* s, uint32_t n, int64_t& out) {
  uint32_t i = 0;
  const bool neg = n > 0 && s[0] == '-';
  if (neg) i = 1;
  uint32_t dot = i;
  while (dot < n && s[dot] != '.') dot++;
  if (dot == n || dot == i) return false;
  const uint32_t fl = n - dot - 1;
  if (fl == 0 || fl > 4) return false;
  uint64_t ip = 0;
  bool big = false;
  for (uint32_t k = i; k < dot; k++) {
    if (!dev_digit(s[k])) return false;
    if (ip > (~0ull - 9) / 10) big = true;  // beyond 2^64: out of range whatever follows
    else ip = ip * 10 + (s[k] - '0');
  }
  uint64_t fp = 0;
  for (uint32_t k = dot + 1; k < n; k++) {
    if (!dev_digit(s[k])) return false;
    fp = fp * 10 + (s[k] - '0');
  }
  for (uint32_t k = fl; k < 4; k++) fp *= 10;
  const uint64_t lim = neg ? (1ull << 63) : (1ull << 63) - 1;
  if (big || ip > (lim - fp) / 10000) return false;
  const uint64_t mag = ip * 10000 + fp;
  if (mag > lim) return false;
  out = neg ? (int64_t)(0 - mag) : (int64_t)mag;
  return true;
}
__device__ bool dev_parse_ipv4(const uint8_t* s, uint32_t n, uint32_t& a) {
  uint32_t i = 0;
  a = 0;
  for (uint32_t part = 0; part < 4; part++) {
    if (i >= n || !dev_digit(s[i])) return false;
    uint32_t v = 0;
    const uint32_t st = i;
    while (i < n && dev_digit(s[i])) {
      v = v * 10 + (s[i] - '0');
      i++;
      if (v > 255) return false;
    }
    if (i - st > 1 && s[st] == '0') return false;  // no leading zeros
    a = (a << 8) | v;
    if (part < 3) {
      if (i >= n || s[i] != '.') return false;
      i++;
    }
  }
  return i == n;
}
__device__ bool dev_parse_ipv6(const uint8_t* s, uint32_t n, uint32_t* w4) {
  uint32_t head[8], tail[8], nh = 0, nt = 0;
  bool dbl = false, v4tail = false, in_tail = false;
  uint32_t v4 = 0, i = 0;
  if (n >= 2 && s[0] == ':' && s[1] == ':') { dbl = true; in_tail = true; i = 2; }
  while (i < n) {
    uint32_t j = i;
    bool dot = false;
    while (j < n && s[j] != ':') { dot = dot || s[j] == '.'; j++; }
    if (dot) {
      if (j != n || !dev_parse_ipv4(s + i, j - i, v4)) return false;
      v4tail = true;
      i = j;
      break;
    }
    if (j == i || j - i > 4) return false;
    uint32_t g = 0;
    for (uint32_t k = i; k < j; k++) {
      const int h = dev_hex(s[k]);
      if (h < 0) return false;
      g = (g << 4) | (uint32_t)h;
    }
    if (in_tail) { if (nt >= 8) return false; tail[nt++] = g; }
    else { if (nh >= 8) return false; head[nh++] = g; }
    if (j == n) { i = j; break; }
    if (j + 1 < n && s[j + 1] == ':') {
      if (dbl) return false;
      dbl = true;
      in_tail = true;
      i = j + 2;
      if (i == n) break;
    } else {
      i = j + 1;
      if (i == n) return false;
    }
  }
  const uint32_t groups = nh + nt + (v4tail ? 2u : 0u);
  if (groups > 8 || (!dbl && groups != 8) || (dbl && groups == 8)) return false;
  uint32_t w[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (uint32_t k = 0; k < nh; k++) w[k] = head[k];
  const uint32_t ts = 8 - nt - (v4tail ? 2u : 0u);
  for (uint32_t k = 0; k < nt; k++) w[ts + k] = tail[k];
  if (v4tail) { w[6] = v4 >> 16; w[7] = v4 & 0xFFFFu; }
  for (uint32_t k = 0; k < 4; k++) w4[k] = (w[2 * k] << 16) | w[2 * k + 1];
  return true;
}
// [v6 | prefix << 8, a0..a3] (image.h T_IP)
__device__ bool dev_parse_ip(const uint8_t* s, uint32_t n, uint32_t* out) {
  uint32_t sl = 0;
  while (sl < n && s[sl] != '/') sl++;
  int prefix = -1;
  if (sl < n) {
    const uint32_t pl = n - sl - 1;
    if (pl == 0 || pl > 3) return false;
    if (pl > 1 && s[sl + 1] == '0') return false;
    prefix = 0;
    for (uint32_t k = sl + 1; k < n; k++) {
      if (!dev_digit(s[k])) return false;
      prefix = prefix * 10 + (int)(s[k] - '0');
    }
  }
  bool v6 = false;
  for (uint32_t k = 0; k < sl; k++) v6 = v6 || s[k] == ':';
  uint32_t a[4] = {0, 0, 0, 0};
  if (v6) {
    if (!dev_parse_ipv6(s, sl, a) || prefix > 128) return false;
  } else {
    if (!dev_parse_ipv4(s, sl, a[0]) || prefix > 32) return false;
  }
  out[0] = (v6 ? 1u : 0u) | ((uint32_t)(prefix < 0 ? (v6 ? 128 : 32) : prefix) << 8);
  for (uint32_t k = 0; k < 4; k++) out[1 + k] = a[k];
  return true;
}

__device__ __forceinline__ void run_bytecode(const Ctx& c, const uint32_t* code, uint32_t n_ins, uint32_t sb, bool& run,
                                             bool& err, Err& e) {
  uint32_t a0 = 0, a1 = 0, a2 = 0, a3 = 0, a4 = 0, a5 = 0, a6 = 0, a7 = 0;
  uint32_t b0 = 0, b1 = 0, b2 = 0, b3 = 0, b4 = 0, b5 = 0, b6 = 0, b7 = 0;
  uint32_t c0 = 0, c1 = 0, c2 = 0, c3 = 0, c4 = 0, c5 = 0, c6 = 0, c7 = 0;
  uint32_t skip = 0;
  for (uint32_t pc = 0; pc < n_ins;) {
    const bool on = run && skip <= pc;
    if (__ballot(on) == 0) {
      const uint32_t nxt = wave_min(run ? skip : 0xFFFFFFFFu);
      if (nxt >= n_ins) break;
      pc = nxt;
      continue;
    }
    const uint2 ins = *reinterpret_cast<const uint2*>(code + 2 * pc);
    const uint32_t w0 = uni(ins.x);
    const uint32_t imm = uni(ins.y);
    const uint32_t op = w0 & 0xFF, D = (w0 >> 8) & 63, A = (w0 >> 14) & 63, B = (w0 >> 20) & 63, C = w0 >> 26;
    if (on) {
      RV va, vb{0, 0, 0};
      CG_SLOT_GET(A, va);
      if (op != OP_RECPUT) CG_SLOT_GET(B, vb);  // RECPUT keeps a position in b
      RV out = va;
      bool wr = true;
      switch (op) {
        case OP_LDV:  // principal / action / resource (their UIDs, from the row), context
          out = imm < 3 ? RV{mk_w0(T_ENT, pick3(imm, c.pt, c.at, c.rt)), pick3(imm, c.pi, c.ai, c.ri), 0}
                        : RV{c.blk[RH_CTX], c.blk[RH_CTX + 1], 0};
          break;
        case OP_LDC: out = load_val(c, c.cpool[imm], c.cpool[imm + 1]); break;
        case OP_LDB: out = mk_bool(imm != 0); break;
        case OP_LDS: out = RV{mk_w0(T_STR, 0), imm, 0}; break;
        case OP_HOT: {
          const uint2 hv = hot_get(c, C);
          if (hot_ok(hv)) { out = load_val(c, hv.x, hv.y); break; }
          hot_err(c, C, hv, e);
          err = true;
          wr = false;
          break;
        }
        case OP_HOTHAS: {
          const uint2 hv = hot_get(c, C);
          const uint32_t q = hot_has(hv);
          if (q == 2u) { hot_err(c, C, hv, e); err = true; wr = false; break; }
          out = mk_bool(q == 1u);
          break;
        }
        case OP_ATTR:
        case OP_HAS: {
          const uint32_t t = tag_of(va);
          const bool has = op == OP_HAS;
          if (t == T_ENT) {
            const uint32_t et = va.w0 & X_MASK, ei = va.w1;
            const uint32_t idx = find_ent(c, et, ei);
            if (idx == NO_ENT) {
              if (has) { out = mk_bool(false); break; }
              e.code = E_ENTITY_MISSING; e.et = et; e.ei = ei; err = true; wr = false;
              break;
            }
            const uint32_t* row = ent_row(c, idx);
            RV got;
            const bool f = rec_get(c, RV{row[ER_ATTR0], row[ER_ATTR1], 0}, imm, got);
            if (has) { out = mk_bool(f); break; }
            if (!f) { e.code = E_ATTR_ENTITY; e.k = imm; e.et = et; e.ei = ei; err = true; wr = false; break; }
            out = got;
          } else if (t == T_REC) {
            RV got;
            const bool f = rec_get(c, va, imm, got);
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
          const bool q = veq(c, va, vb, deep);
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
            const RV x = load_val(c, rd(c, ref, 1 + 2 * k), rd(c, ref, 2 + 2 * k));
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
          out = mk_bool(like_match(c, va.w1, c.cpool + imm));
          break;
        case OP_CONTAINS: {
          if (tag_of(va) != T_SET) { type_err(e, TN_SET, va); err = true; wr = false; break; }
          const uint32_t ref = va.w0 & X_MASK, n = va.w1;
          bool deep = false, f = false;
          for (uint32_t k = 0; k < n && !f; k++) f = veq(c, load_val(c, rd(c, ref, 1 + 2 * k), rd(c, ref, 2 + 2 * k)), vb, deep);
          if (deep) { e.code = E_DEPTH; err = true; wr = false; break; }
          out = mk_bool(f);
          break;
        }
        case OP_CALL: {
          if (C == CO_PARSE_IP || C == CO_PARSE_DEC) {  // ip(x) / decimal(x) into lane scratch at imm
            const uint32_t which = C == CO_PARSE_DEC ? 1u : 0u;
            if (tag_of(va) != T_STR) { e.code = E_EXT_ARG; e.aux = which; err = true; wr = false; break; }
            const uint8_t* sp;
            uint32_t sn;
            str_span(c, va.w1, sp, sn);
            bool ok;
            if (which) {
              int64_t x = 0;
              ok = dev_parse_decimal(sp, sn, x);
              if (ok) { c.lh[imm] = (uint32_t)((uint64_t)x & 0xFFFFFFFFu); c.lh[imm + 1] = (uint32_t)((uint64_t)x >> 32); }
            } else {
              ok = dev_parse_ip(sp, sn, c.lh + imm);
            }
            if (!ok) { e.code = E_EXT_PARSE; e.aux = which; e.k = va.w1; err = true; wr = false; break; }
            out = RV{mk_w0(which ? T_DEC : T_IP, mk_ref(SP_LANE, imm)), 0, 0};
            break;
          }
          if (C == CO_CONTAINS_ALL || C == CO_CONTAINS_ANY || C == CO_IS_EMPTY) {
            if (tag_of(va) != T_SET) { type_err(e, TN_SET, va); err = true; wr = false; break; }
            if (C == CO_IS_EMPTY) { out = mk_bool(va.w1 == 0); break; }
            if (tag_of(vb) != T_SET) { type_err(e, TN_SET, vb); err = true; wr = false; break; }
            const uint32_t ra = va.w0 & X_MASK, na = va.w1, rb = vb.w0 & X_MASK, nb = vb.w1;
            bool deep = false;
            bool all = true, any = false;
            for (uint32_t j = 0; j < nb; j++) {
              const RV y = load_val(c, rd(c, rb, 1 + 2 * j), rd(c, rb, 2 + 2 * j));
              bool f = false;
              for (uint32_t i = 0; i < na && !f; i++) f = veq(c, load_val(c, rd(c, ra, 1 + 2 * i), rd(c, ra, 2 + 2 * i)), y, deep);
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
          const uint32_t off = imm & 0xFFFFFu, n = imm >> 20;
          c.lh[off] = n;
          out = RV{mk_w0(op == OP_SETNEW ? T_SET : T_REC, mk_ref(SP_LANE, off)), n, 0};
          break;
        }
        case OP_SETPUT:
        case OP_RECPUT: {
          // store slot A (register form) into the container in slot D at position pos (SETPUT:
          // imm; RECPUT: c | b << 6, imm = key)
          wr = false;
          RV cont;
          CG_SLOT_GET(D, cont);
          const uint32_t base = cont.w0 & OFF_MASK, n = cont.w1;
          const bool isrec = op == OP_RECPUT;
          const uint32_t stride = isrec ? 3u : 2u;
          const uint32_t pos = isrec ? (C | (B << 6)) : imm;
          uint32_t* slotp = c.lh + base + 1 + stride * pos;
          if (isrec) *slotp++ = imm;
          if (tag_of(va) == T_LONG) {
            const int64_t x = as_i64(va);
            if (x >= INT32_MIN && x <= INT32_MAX) { slotp[0] = mk_w0(T_LONG, 0); slotp[1] = va.w1; }
            else {
              const uint32_t sp = base + 1 + stride * n + 2 * pos;
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
      if (wr) CG_SLOT_SET(D, out);
    }
    pc++;
  }
}

// ---- the kernel -----------------------------------------------------------------------------
constexpr uint32_t CAPR_L = 8;  // reasons per lane staged in LDS before spilling to global

// GLANE: lane scratch in the batch's global lane area (a.lane, lane_stride words per request)
// instead of a private array, for images whose bytecode needs more than LANE_WORDS.
template <bool BYTECODE, bool GLANE = false>
__global__ __launch_bounds__(BLOCK) void cedar_eval_kernel(KArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t chunk_lds[CHUNK_WORDS];  // staged policy records
  // per-lane reason lists of the current tier ([forbid|permit][slot][lane]); global stores inside
  // the policy loop would serialise later heap loads behind them (in-order vmcnt)
  __shared__ uint32_t rsn_lds[2 * CAPR_L * BLOCK];
  extern __shared__ uint2 hot_lds[];                                          // [n_hot][BLOCK]
  const uint32_t gid = blockIdx.x * BLOCK + threadIdx.x;
  const uint32_t n_req = a.n_dev ? min(*a.n_dev, a.n_req) : a.n_req;  // follow-up: count on the device
  if (blockIdx.x * BLOCK >= n_req) return;  // (block-uniform: a follow-up's unused blocks stage no policy)
  const bool valid = gid < n_req;
  // position p in the first pass's launch order (first pass: gid; follow-up: its worklist entry's),
  // the request's row r (ord[p] for a batch grouped on the device); the result slot is the worklist
  // entry, or the position
  const uint32_t p = valid ? (a.req_idx ? a.req_idx[gid] : gid) : 0;
  const uint32_t r = valid ? (a.ord ? a.ord[p] : p) : 0;
  const uint32_t wo = a.req_idx ? gid : p;

  uint32_t lane_scratch[GLANE ? 1 : LANE_WORDS];
  Ctx c;
  const uint32_t* rowp = a.rows + (size_t)r * a.row_words;
  c.blk = a.heap + (valid ? rowp[RW_BLK] : 0);  // (the row's block offset: no req_base upload)
  c.cpool = a.cpool;
  c.lh = GLANE ? a.lane + (size_t)(valid ? gid : 0) * a.lane_stride : lane_scratch;
  c.hot = a.hot;
  c.gstr_off = a.gstr_off;
  c.gstr_bytes = a.gstr_bytes;
  c.bstr_off = a.bstr_off;
  c.bstr_bytes = a.bstr_bytes;
  c.n_gstr = a.n_gstr;
  c.hotl = hot_lds + threadIdx.x;
  c.hstride = BLOCK;
  c.srows = a.srows;
  c.shash = a.shash;
  c.n_static = a.n_static;
  c.smask = a.smask;
  c.pb0 = c.pb1 = c.pb2 = c.pb3 = 0;
  c.rb0 = c.rb1 = c.rb2 = c.rb3 = 0;
  c.p_anc = c.p_nanc = c.r_anc = c.r_nanc = 0;
  c.p_base = c.r_base = c.blk;
  c.a_anc = c.a_nanc = 0;
  uint32_t am0 = 0, am1 = 0;  // action mask over the image action table: action in act[k]
  uint32_t as0 = 0, as1 = 0;  // action == act[k]
  if (valid) {
    c.nent = c.blk[RH_NENT];
    c.pt = rowp[RW_P]; c.pi = rowp[RW_P + 1];
    c.at = rowp[RW_A]; c.ai = rowp[RW_A + 1];
    c.rt = rowp[RW_R]; c.ri = rowp[RW_R + 1];
    c.pidx = c.blk[RH_PIDX]; c.aidx = c.blk[RH_AIDX]; c.ridx = c.blk[RH_RIDX];
    anc_of(c, c.pidx, c.p_base, c.p_anc, c.p_nanc);
#define CG_ANC(k) \
    c.t##k = k < c.p_nanc ? c.p_base[c.p_anc + 2 * k] : 0xFFFFFFFFu; \
    c.i##k = k < c.p_nanc ? c.p_base[c.p_anc + 2 * k + 1] : 0xFFFFFFFFu;
    CG_ANC(0) CG_ANC(1) CG_ANC(2) CG_ANC(3) CG_ANC(4) CG_ANC(5) CG_ANC(6) CG_ANC(7)
#undef CG_ANC
    anc_of(c, c.ridx, c.r_base, c.r_anc, c.r_nanc);
    // ancestor-or-self Bloom filters of principal and resource
    bloom_add(c.pb0, c.pb1, c.pb2, c.pb3, uid_bloom_bit(c.pt, c.pi));
    for (uint32_t k = 0; k < c.p_nanc; k++)
      bloom_add(c.pb0, c.pb1, c.pb2, c.pb3, uid_bloom_bit(c.p_base[c.p_anc + 2 * k], c.p_base[c.p_anc + 2 * k + 1]));
    bloom_add(c.rb0, c.rb1, c.rb2, c.rb3, uid_bloom_bit(c.rt, c.ri));
    for (uint32_t k = 0; k < c.r_nanc; k++)
      bloom_add(c.rb0, c.rb1, c.rb2, c.rb3, uid_bloom_bit(c.r_base[c.r_anc + 2 * k], c.r_base[c.r_anc + 2 * k + 1]));
  } else {
    c.nent = 0; c.pt = c.pi = c.at = c.ai = c.rt = c.ri = 0xFFFFFFFFu;
    c.t0 = c.t1 = c.t2 = c.t3 = c.t4 = c.t5 = c.t6 = c.t7 = 0xFFFFFFFFu;
    c.i0 = c.i1 = c.i2 = c.i3 = c.i4 = c.i5 = c.i6 = c.i7 = 0xFFFFFFFFu;
    c.pidx = c.aidx = c.ridx = NO_ENT;
  }
  if (a.amask_ok) {
    uint32_t a_off = 0, a_n = 0;
    const uint32_t* a_base = c.blk;
    if (valid) anc_of(c, c.aidx, a_base, a_off, a_n);
    const uint32_t n_act = a.n_act;
    for (uint32_t k = 0; k < n_act; k++) {
      const uint32_t qt = uni(a.act[2 * k]), qi = uni(a.act[2 * k + 1]);
      const bool self = valid && c.at == qt && c.ai == qi;
      const bool hit = self || (valid && a_n && anc_scan(a_base, a_off, a_n, qt, qi));
      if (hit) { if (k < 32) am0 |= 1u << k; else am1 |= 1u << (k - 32); }
      if (self) { if (k < 32) as0 |= 1u << k; else as1 |= 1u << (k - 32); }
    }
  }
  // hot attribute paths (resolved by the encoder into the request row) into LDS
  {
    const uint32_t* row = a.rows + (size_t)r * a.row_words;
    for (uint32_t h = 0; h < a.n_hot; h++)
      c.hotl[h * c.hstride] = valid ? make_uint2(row[RW_HDR + 2 * h], row[RW_HDR + 2 * h + 1]) : make_uint2(0u, 0u);
    c.rowx = (valid && a.hlists) ? row + RW_HDR + 2 * a.n_hot : nullptr;
    c.lmask = a.hlists;
  }

  bool decided = !valid;
  uint32_t cbeg = 0;
  const uint32_t n_tiers = a.n_tiers;
  for (uint32_t t = 0; t < n_tiers; t++) {
    const uint32_t cend = uni(a.tier_cend[t]);
    uint32_t nf = 0, np = 0, ne = 0;
    for (uint32_t ch = cbeg; ch < cend; ch++) {
      // stage the chunk's policy records in LDS (block-cooperative, coalesced 16-byte loads); a
      // record too large for LDS has a chunk of its own and is read in place (CHUNK_GLOBAL)
      const uint32_t c_off = uni(a.chunks[4 * ch]), c_nw = uni(a.chunks[4 * ch + 1]);
      const uint32_t c_p0 = uni(a.chunks[4 * ch + 2]), c_p1 = uni(a.chunks[4 * ch + 3]);
      const bool glob = (c_nw & CHUNK_GLOBAL) != 0;
      if (!__syncthreads_or(!decided)) break;  // whole block decided: later chunks/tiers are moot
      if (!glob) {
        const uint4* src = reinterpret_cast<const uint4*>(a.pstream + c_off);
        uint4* dst = reinterpret_cast<uint4*>(chunk_lds);
        for (uint32_t k = threadIdx.x; k < (c_nw >> 2); k += BLOCK) dst[k] = src[k];
      }
      __syncthreads();
      if (__ballot(!decided) == 0) continue;  // this wave is done; keep joining the barriers
      // the chunk's policies; `base` is the LDS copy or, for CHUNK_GLOBAL, the stream itself (two
      // inlined copies, each with its own address space)
      auto run_chunk = [&](const uint32_t* base) {
      uint32_t rw = 0;                         // record offset inside the chunk (words)
      for (uint32_t p = c_p0; p < c_p1; p++) {
        const uint32_t* rec = base + rw;
        const uint4* d4 = reinterpret_cast<const uint4*>(rec);
        const uint4 q0 = d4[0], q1 = d4[1], q2 = d4[2], q3 = d4[3];
        const uint32_t flags = uni(q0.x), kinds = uni(q0.y);
        const uint32_t p_ty = uni(q0.z), p_et = uni(q0.w), p_ei = uni(q1.x);
        const uint32_t a_et = uni(q1.y), a_ei = uni(q1.z);
        const uint32_t r_ty = uni(q1.w), r_et = uni(q2.x), r_ei = uni(q2.y);
        const uint32_t n_code = uni(q2.w), n_atom = uni(q3.x), n_lane = uni(q3.y);
        const uint32_t am0p = uni(q3.z), am1p = uni(q3.w);
        rw += (POL_WORDS + n_code + 3) & ~3u;
        const uint32_t pk = kinds & 0xFF, ak = (kinds >> 8) & 0xFF, rk = (kinds >> 16) & 0xFF;
        bool ok = !decided;
        // action scope: one AND against the per-request action mask
        if (ak != SK_ANY) {
          if (a.amask_ok) {  // `==` tests the action itself, `in` its ancestors too
            ok = ok && (ak == SK_EQ ? (((as0 & am0p) | (as1 & am1p)) != 0) : (((am0 & am0p) | (am1 & am1p)) != 0));
          } else if (ak == SK_EQ) {
            ok = ok && c.at == a_et && c.ai == a_ei;
          } else if (ak == SK_IN) {
            ok = ok && ((c.at == a_et && c.ai == a_ei) || anc_has(c, c.aidx, a_et, a_ei));
          } else {
            bool any = false;
            for (uint32_t k = 0; k < a_et; k++) {
              const uint32_t qt = uni(a.cpool[a_ei + 2 * k]), qi = uni(a.cpool[a_ei + 2 * k + 1]);
              any = any || (c.at == qt && c.ai == qi) || anc_has(c, c.aidx, qt, qi);
            }
            ok = ok && any;
          }
        }
        // principal scope (type test, then Bloom-gated ancestor test)
        if (pk == SK_IS || pk == SK_ISIN) ok = ok && c.pt == p_ty;
        if (pk == SK_EQ) ok = ok && c.pt == p_et && c.pi == p_ei;
        else if (pk == SK_IN || pk == SK_ISIN) ok = ok && p_in(c, p_et, p_ei, (flags >> 16) & 0x7F);
        // resource scope
        if (rk == SK_IS || rk == SK_ISIN) ok = ok && c.rt == r_ty;
        if (rk == SK_EQ) ok = ok && c.rt == r_et && c.ri == r_ei;
        else if (rk == SK_IN || rk == SK_ISIN) ok = ok && r_in(c, r_et, r_ei, (flags >> 24) & 0x7F);
        if (__ballot(ok) == 0) continue;

        // ---- conditions ----
        bool run = ok;
        bool err = false;
        Err e{0, 0, 0, 0, 0};
        if (flags & PF_ATOMIC) {
          // atom graph: each lane follows its own forward path; atom i runs for the lanes at i
          const uint32_t na = n_atom / ATOM_WORDS;
          uint32_t pc = run ? (na ? 0u : AT_SAT) : AT_UNSAT;
          for (;;) {
            const uint32_t i = wave_min(pc < na ? pc : 0xFFFFFFFFu);
            if (i >= na) break;
            const uint4 at = *reinterpret_cast<const uint4*>(rec + POL_WORDS + ATOM_WORDS * i);
            const uint32_t w0 = uni(at.x), w1 = uni(at.y), w2 = uni(at.z), w3 = uni(at.w);
            if (pc == i) {
              const uint32_t rr = eval_atom<true>(c, rec, w0 & 0xFF, (w0 >> 8) & 0xFF, w1, w2, w3, e);
              if (rr == 2u) { err = true; pc = AT_UNSAT; }
              else pc = rr ? ((w0 >> 16) & 0xFF) : (w0 >> 24);
            }
          }
          run = pc == AT_SAT;
        } else if constexpr (BYTECODE) {
          // spilled registers (slots 8..) sit at the end of the policy's lane area
          const uint32_t sb = n_atom > NSLOT ? n_lane - 3 * (n_atom - NSLOT) : 0u;
          run_bytecode(c, rec + POL_WORDS, n_code >> 1, sb, run, err, e);
        }
        // ---- record outcome ----
        if (ok) {
          if (err) {
            if (ne < a.cape) {
              uint32_t* er = a.errs + ((size_t)wo * a.cape + ne) * ERR_WORDS;
              er[0] = p; er[1] = e.code | (e.aux << 8); er[2] = e.k; er[3] = e.et; er[4] = e.ei; er[5] = 0;
            }
            ne++;
          } else if (run) {
            if (flags & PF_FORBID) {
              if (nf < CAPR_L) rsn_lds[nf * BLOCK + threadIdx.x] = p;
              else if (nf < a.capr) a.reasons_f[(size_t)wo * a.capr + nf] = p;
              nf++;
            } else {
              if (np < CAPR_L) rsn_lds[(CAPR_L + np) * BLOCK + threadIdx.x] = p;
              else if (np < a.capr) a.reasons_p[(size_t)wo * a.capr + np] = p;
              np++;
            }
          }
        }
      }
      };
      if (glob) run_chunk(a.pstream + c_off);
      else run_chunk(chunk_lds);
    }
    if (!decided) {
      if (t + 1 == n_tiers || nf || np || ne) {
        const uint32_t dec = nf ? DEC_DENY : (np ? DEC_ALLOW : DEC_DENY);
        const uint32_t nr = nf ? nf : np;
        uint32_t fl = RF_VALID | (nf ? RF_FORBID : 0u);
        if (nr > a.capr || ne > a.cape) fl |= RF_OVERFLOW;
        // flush the LDS-staged reasons of the deciding list
        const uint32_t nflush = min(min(nr, a.capr), CAPR_L);
        uint32_t* dst = (nf ? a.reasons_f : a.reasons_p) + (size_t)wo * a.capr;
        const uint32_t lbase = nf ? 0u : CAPR_L;
        for (uint32_t k = 0; k < nflush; k++) dst[k] = rsn_lds[(lbase + k) * BLOCK + threadIdx.x];
        a.res[2 * (size_t)wo] = dec | (t << 8) | (fl << 16);
        a.res[2 * (size_t)wo + 1] = min(nr, 0xFFFFu) | (min(ne, 0xFFFFu) << 16);
        decided = true;
      }
    }
    cbeg = cend;
  }
}


// ---- probe kernel: request-per-wave over the two-level scope / attribute index -----------------
// One wave evaluates one request (image.h "scope index"):
//   1. the request row (UIDs, ancestor-list offsets, hot paths pre-resolved by the encoder) is
//      read with wave-uniform loads; lanes copy the hot values into LDS;
//   2. lane k probes the level-1 table for (principal, action, resource) key k: for every key
//      combo the image uses, the product of the request's candidate components (ancestor-or-self
//      UIDs, type, wildcard); then level 2 under each found key for the hot slots in its hmask,
//      with the request's own value of that slot;
//   3. the found buckets' candidate heads (descriptor + first atoms, 128 B, in bucket order) run
//      one per lane: cheap scope re-check, then the lane's atom graph;
//   4. satisfied / erroring candidates are collected in LDS and merged into policy order with the
//      deciding tier, duplicates removed, as the stream kernel writes them.
// Structural (set / record) equality is left to the stream kernel: such a request is flagged
// RF_OVERFLOW and the host re-runs it there (rare: templates compare primitives).
constexpr uint32_t WAVES = BLOCK / 64;

__device__ __forceinline__ uint32_t mbcnt64(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
__device__ __forceinline__ uint32_t popc64(uint64_t m) { return (uint32_t)__popcll(m); }
// LDS written by some lanes of this wave, then read by others
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// inclusive prefix sum across the wave
__device__ __forceinline__ uint32_t wave_scan(uint32_t x, uint32_t lane) {
  for (uint32_t o = 1; o < 64; o <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)x, o);
    if (lane >= o) x += y;
  }
  return x;
}

// bucket words in LDS: first head index | key combo << EF_COMBO (the image keeps heads below 2^27)
constexpr uint32_t EF_COMBO = 27, EF_FIRST = (1u << EF_COMBO) - 1u;
// the pooled candidate pass's staged prefixes: exclusive candidate prefix | segment << FP_SEG (a
// round's candidates stay below 2^24: its requests hold <= KArgs::scan_heavy heads each), and the
// list pairs it stages per round
constexpr uint32_t FP_SEG = 24, FP_PRE = (1u << FP_SEG) - 1u, FLAT_PAIRS = 128;
// segments with a FLAT state region (only the 8-lane candidate pass uses it)
constexpr uint32_t FLAT_NS(uint32_t seg) { return seg == 8 ? 8u : 1u; }
// Per-wave LDS of the probe kernel, one region per request segment of SEG lanes.
// SLIM (one-request waves, images of <= RANK_POL policies): no hm; a hit's kind, tier and error
// slot ride in its hp word (SLIM_* below), so the large stage's wave takes 8,960 B of LDS.
// HOTC: hot entries per request row (the compact candidate pass: images of <= 16 hot values and
// staged like words).
template <uint32_t SEG, uint32_t HCAP, bool SLIM = false, uint32_t HOTC = NHOT>
struct alignas(16) SegLds {  // (16: the counting merge reads hp four words at a time)
  static constexpr uint32_t NS = 64 / SEG;     // requests per wave
  // staged buckets per request (>= 2 stages; the compact candidate pass stages 16 at a time)
  static constexpr uint32_t EC = SEG >= 32 ? 2 * SEG : (HOTC < NHOT ? 16 : 32);
  static constexpr uint32_t HC = HCAP;         // hits per request (more: RF_BIG / RF_GENERAL re-run)
  // error details per request (more: the on-device follow-up, which holds 32; more still: the
  // stream kernel). 32 keeps the large stage's 4-wave block under 53 KB: 3 blocks per CU
  static constexpr uint32_t XC = HCAP >= 256 ? 32 : 8;
  // Rows are not padded off the 64 LDS banks: the segments of a wave that touch element j of their
  // rows in lockstep conflict (SQ_LDS_BANK_CONFLICT is ~1/3 of SQ_LDS_IDX_ACTIVE here), but those
  // cycles are ~0.3 % of the kernel's wave cycles, and one padding word per row would take the
  // 4-wave SPLIT candidate pass from 10,240 to 10,496 B per block, past 16 blocks per CU.
  static constexpr uint32_t PAD = 0;
  // the staged buckets live until the key loop ends, the merge's sort keys only after it: one region
  union {
    struct {
      uint32_t efirst[NS][EC + PAD];   // found bucket: first head index | key combo << EF_COMBO
      uint32_t epre[NS][EC + PAD];     // candidate counts, then their exclusive prefix
    } b;
    uint32_t hs[NS][HC + PAD];         // merge: sort keys (policy index << 12 | hit slot)
  } u;
  uint32_t hp[NS][HC + PAD];       // hit: global policy index
  uint32_t hm[NS][SLIM ? 1 : HC + PAD];  // hit: kind (0 permit, 1 forbid, 2 error) | tier << 8 | error slot << 16
  uint32_t he[NS][XC * 4 + PAD];   // error details: code | aux << 8, k, et, ei
  // (hot rows one uint2 longer: the pooled candidate pass reads slot h of several requests' rows in
  // lockstep, which unpadded rows (64 words apart) put on the same banks)
  uint2 hot[NS][HOTC + (NS > 1 ? 1 : 0)];
  // the candidate pass's wave-wide task pool (FLAT: SPLIT, 8-lane segments): every segment's request
  // context, for lanes that evaluate another segment's candidates, and its running state (rows of
  // 5 uint4, the last unused: 80 bytes apart, 8 requests' rows on disjoint banks)
  uint4 cx[FLAT_NS(SEG)][FLAT_NS(SEG) > 1 ? 5 : 4];  // (blk, pt, pi, at), (ai, rt, ri, p_anc), (r_anc, a_anc, nanc p|r, a_nanc | self << 16), (rowo, am lo, am hi, 0)
  uint32_t sst[FLAT_NS(SEG)][4];   // hits recorded, error details, lowest tier with a hit, flags (1: structural)
  uint32_t sne[FLAT_NS(SEG)];      // buckets staged
  // the compact pooled candidate pass: each lane's candidate's head atoms (the head's second 64
  // bytes, loaded with its descriptor), [atom][lane], so the atom loop reads LDS, not memory
  static constexpr bool ATOMS = NS == 8 && HOTC < NHOT;
  uint4 at4[ATOMS ? HEAD_ATOMS : 1][ATOMS ? 64 : 1];
};

// Slim per-request context of the probe kernel (everything wave-uniform but the pointers' data).
struct PCtx {
  const uint32_t* blk;
  const uint32_t* cpool;
  uint32_t* lh;
  const uint32_t* gstr_off;
  const uint8_t* gstr_bytes;
  const uint32_t* bstr_off;
  const uint8_t* bstr_bytes;
  uint32_t n_gstr;
  uint2* hotl;
  static constexpr uint32_t hstride = 1;
  uint32_t pt, pi, at, ai, rt, ri;
  uint32_t p_anc, p_nanc, r_anc, r_nanc, a_anc, a_nanc;
  // the row's element-hash list offsets per hot slot: rowb[rowo + h] (rowb launch-uniform, so the
  // per-request part is one 32-bit word: a 64-bit pointer here was the candidate pass's spill)
  const uint32_t* rowb;
  uint32_t rowo;  // 0xFFFFFFFF: none
  uint32_t lmask;  // the list slots (KArgs::hlists): slot h's word at its rank among them
  __device__ uint32_t hlist(uint32_t h) const {
    return (rowo != 0xFFFFFFFFu && ((lmask >> h) & 1u)) ? rowb[rowo + __popc(lmask & ((1u << h) - 1u))] : 0xFFFFFFFFu;
  }
  uint32_t lkb, lslot;  // like words staged at hot index lkb (0xFFFFFFFF: not), like slots (KArgs)
};

// X in (qt, qi) for X with UID (st, si) and ancestor pairs at blk[off + 2k]
__device__ __forceinline__ bool anc_in(const uint32_t* blk, uint32_t off, uint32_t n, uint32_t st, uint32_t si,
                                       uint32_t qt, uint32_t qi) {
  return (st == qt && si == qi) || anc_scan(blk, off, n, qt, qi);
}
__device__ __forceinline__ bool var_in(const PCtx& c, uint32_t h, uint32_t qt, uint32_t qi, uint32_t) {
  if (h == 0) return anc_in(c.blk, c.p_anc, c.p_nanc, c.pt, c.pi, qt, qi);
  if (h == 2) return anc_in(c.blk, c.r_anc, c.r_nanc, c.rt, c.ri, qt, qi);
  return anc_in(c.blk, c.a_anc, c.a_nanc, c.at, c.ai, qt, qi);
}

// One (principal, action, resource) component: kind KC_*, list index j of the request's
// ancestor-or-self list (j = 0: the UID itself, j > 0: ancestor j - 1)
__device__ __forceinline__ uint2 key_comp(uint32_t kc, uint32_t j, uint32_t st, uint32_t si, const uint32_t* blk,
                                          uint32_t off) {
  if (kc == KC_WILD) return make_uint2(KW_ANY, KW_ANY);
  if (kc == KC_TYPE) return make_uint2(st, KW_ANY);
  const uint32_t* l = blk + (int32_t)off;  // (signed: image.h "ancestor lists")
  return j ? make_uint2(__builtin_nontemporal_load(l + 2 * (j - 1)), __builtin_nontemporal_load(l + 2 * (j - 1) + 1))
           : make_uint2(st, si);
}

// key filter: false = the key is certainly absent from the scope index
__device__ __forceinline__ bool filt_maybe(const uint32_t* bfilt, uint32_t fmask, uint32_t hash) {
  const uint2 w = *reinterpret_cast<const uint2*>(bfilt + 2 * (size_t)(hash & fmask));
  const uint64_t need = filt_need(hash);
  return ((((uint64_t)w.y << 32) | w.x) & need) == need;
}

// probe: (first, count, hmask) of the slot matching key words w0..w6 (+ v0, v1 for level 2)
// (level-1 probes also return the entry's level-2 bloom in *bloom and its cmask in *cmask)
template <bool ST = false>
__device__ __forceinline__ uint3 probe(const uint32_t* btab, uint32_t bmask, uint32_t hash, uint32_t w0, uint2 p, uint2 q,
                                       uint2 r, uint32_t v0, uint32_t v1, uint32_t& steps, uint4* bloom = nullptr,
                                       uint32_t* cmask = nullptr, uint32_t split = 0) {
  uint32_t h = hash & bmask;
  for (;;) {
    if (ST) steps++;
    const uint4* sl = reinterpret_cast<const uint4*>(btab + (size_t)h * BT_WORDS);
    if (split) {  // an empty or foreign slot costs one 16-byte load
      const uint4 x = sl[0];
      if (x.x == 0) return make_uint3(0, 0, 0);
      if (x.x == w0 && x.y == p.x && x.z == p.y && x.w == q.x) {
        const uint4 y = sl[1], z = sl[2];
        if (y.x == q.y && y.y == r.x && y.z == r.y && (!(w0 & BT_L2) || (y.w == v0 && z.x == v1))) {
          if (bloom) *bloom = sl[3];
          if (cmask) *cmask = y.w;
          return make_uint3(z.y, z.z, z.w);
        }
      }
      h = (h + 1) & bmask;
      continue;
    }
    // the whole 64-byte slot in one round trip, compared once every word arrives (7 % faster on
    // C3 than loading the key's first words and the rest on a match: profiles/r02/ab_whole_slot)
    const uint4 x = sl[0], y = sl[1], z = sl[2];
    const uint4 bl = bloom ? sl[3] : make_uint4(0u, 0u, 0u, 0u);
    if (x.x == 0) return make_uint3(0, 0, 0);
    if (x.x == w0 && x.y == p.x && x.z == p.y && x.w == q.x && y.x == q.y && y.y == r.x && y.z == r.y &&
        (!(w0 & BT_L2) || (y.w == v0 && z.x == v1))) {
      if (bloom) *bloom = bl;
      if (cmask) *cmask = y.w;
      return make_uint3(z.y, z.z, z.w);
    }
    h = (h + 1) & bmask;
  }
}
// level-2 key hash h2 possibly under the level-1 entry whose bloom is b
__device__ __forceinline__ bool l2_bloom_maybe(uint4 b, uint32_t h2) {
  const uint32_t bits = l2_bloom_bits(h2);
  bool ok = true;
  for (uint32_t j = 0; j < 3; j++) {
    const uint32_t x = (bits >> (7 * j)) & 127u;
    const uint32_t w = x < 64 ? (x < 32 ? b.x : b.y) : (x < 96 ? b.z : b.w);
    ok = ok && ((w >> (x & 31)) & 1u);
  }
  return ok;
}

// ---- split first pass: the index scan ---------------------------------------------------------
// SEG lanes per request enumerate its level-1 keys as the probe kernel does (every used combo's
// product of candidate components, SEG keys a step) and probe each found entry's level-2 keys
// (hot slots in its hmask, set-membership / prefix list elements in its cmask), segment by
// segment alternating the two; found buckets that hold candidate heads go straight to a.scan. No
// LDS and no candidate evaluation: far fewer registers than the probe kernel, so more requests are
// in flight per CU; the probe kernel's SPLIT variant then evaluates the buckets' heads.
// principal key ancestors the scan stages in LDS per request (more: read from the request block)
constexpr uint32_t SCAN_ANC = 40;
// key-filter pass: keys per lane per round (independent loads in flight), and the filter-passing
// keys a request lists in LDS (more: it probes every key, as with the filter off)
constexpr uint32_t SCAN_PU = 4, SCAN_POS = 64;
// contexts a request looks up in the scope-bitset pass (more: it enumerates every key instead), and
// the flag of a listed key the bitsets found (image.h "scope bitsets")
constexpr uint32_t LIST_EXACT = 0x80000000u, SCAN_POS_B = 40;  // (CTX_CAP: image.h)
constexpr uint32_t SCAN_HOT = 16;  // hot values the scan stages in LDS (the rest read from the row)
static_assert(EQF_SLOTS <= SCAN_HOT, "equality-filter slots are staged in the scan's LDS");
constexpr uint32_t SCAN_ROW = 56;  // scan LDS row words (64 - 8: see s_kid; the LDS stays under 1/24 of a CU for 6 waves per SIMD)
static_assert(SCAN_ANC + 2 <= SCAN_ROW - 1 && SCAN_POS_B + 2 <= SCAN_ROW, "scan LDS rows (s_kid's last word: the presence mask)");
constexpr uint32_t SCAN_PB = 8;    // bit tests per lane per round (loads in flight)
constexpr uint32_t MEMB_U = 4;     // duplicate-class members a lane copies per round (loads in flight)
constexpr uint32_t HM_CLASS = 1u << 24;  // hit-slot word (wl.hm): the slot holds a whole duplicate class
constexpr uint32_t RANK_POL = 16384;  // the large stage's rank pass: policy indices its bitmap covers
// SLIM hit words: policy index (< RANK_POL) | kind << 14 | tier << 16 | error slot << 24
constexpr uint32_t SLIM_KIND = 14, SLIM_TIER = 16, SLIM_SLOT = 24, SLIM_POL = 0x3FFFu;
static_assert(RANK_POL - 1 <= SLIM_POL, "SLIM hit words hold a policy index below RANK_POL");
__device__ __forceinline__ uint32_t nth_bit(uint32_t m, uint32_t k) {  // index of the k-th set bit of m
  for (uint32_t i = 0; i < k; i++) m &= m - 1;
  return m ? (uint32_t)__builtin_ctz(m) : 0u;
}
// combos whose action / resource component keys on the entity (image.h key_combo)
constexpr uint32_t combo_mask_of(uint32_t k, uint32_t shift, uint32_t mask) {
  uint32_t m = 0;
  for (uint32_t cb = 0; cb < 32; cb++)
    if (((cb >> shift) & mask) == k) m |= 1u << cb;
  return m;
}
constexpr uint32_t COMBO_AENT = combo_mask_of(KC_ENT, 2, 1), COMBO_RENT = combo_mask_of(KC_ENT, 3, 3),
                   COMBO_PENT = combo_mask_of(KC_ENT, 0, 3);
// BITS: the variant with the scope-bitset pass (launched when a.scan_filt and the image has
// bitsets); the other one carries none of its registers
// STATS (CEDARGPU_SCAN_STATS=1, profiling): sums over the launch into a.stats[0..15]: [0] requests
// [1] level-1 probes [2] level-1 entries found [3] level-2 probes [4] level-2 buckets found
// [5] loop iterations (per wave) [6] segment iterations spent on level-2 probes [7] segment
// iterations in all [8] prologue cycles [9] loop cycles (per wave, s_memtime) [10] keys enumerated
// LOOKUP (BITS only): the scan looks up the contexts the encoder did not resolve (image.h RH_SCTX)
// in the context table itself; without it such a request enumerates its keys instead, and the
// kernel carries none of the lookup's registers (CEDARGPU_SCAN_LOOKUP=1: with it, A/B)
template <uint32_t SEG, uint32_t MINW = 1, bool BITS = false, bool STATS = false, bool LOOKUP = false>
__global__ __launch_bounds__(64, MINW) void cedar_scan_kernel(KArgs a) {
  const uint64_t t0 = STATS ? clock64() : 0;
  uint32_t st[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  // per request: its first SCAN_ANC key ancestors and its hot values, loaded in one round trip
  // before the key loop (the request block and row are cold: each key step would otherwise start
  // with a dependent HBM load)
  // rows padded off a multiple of the 64 LDS banks: the segments of a wave index them in lockstep
  // (BITS: no UIDs staged: a key the bitsets find is read from svals, no key hash or probe; a
  // request off the bitset path reads its key ancestors from its list)
  constexpr uint32_t ANC_ST = BITS ? 1u : SCAN_ANC;  // principal key ancestors staged (UIDs)
  __shared__ uint2 s_anc[BITS ? 1 : 64 / SEG][ANC_ST + 1];
  __shared__ uint2 s_hot[64 / SEG][SCAN_HOT + 1];  // the first SCAN_HOT hot values
  // BITS: the key-entity index of the principal ([0]) and of each staged key ancestor ([j]: j - 1),
  // the request's contexts (combo | hs << 8, bitset row) and its listed keys
  // (LIST_EXACT | combo << 26 | the bit's rank in svals, or combo << 11 for a type / wildcard
  // principal combo's single key)
  // (rows of SCAN_ROW words: the 8 lanes of each of the 8 segments read consecutive entries at
  // once, so rows 8 banks apart (56 words) take all 64 banks without a conflict)
  __shared__ uint32_t s_kid[BITS ? 64 / SEG : 1][SCAN_ROW];
  // (found contexts: combo and bitset row; 8-byte entries, rows padded off a multiple of the 64
  // banks: the wave's segments read the same context index in lockstep)
  __shared__ uint2 s_cx[BITS ? 64 / SEG : 1][CTX_CAP + 1];
  __shared__ uint32_t s_pos[BITS ? 64 / SEG : 1][SCAN_ROW];
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t seg = lane / SEG, sl = lane % SEG, sbase = seg * SEG;
  const uint64_t smask = SEG == 64 ? ~0ull : (((1ull << SEG) - 1ull) << sbase);
  auto sballot = [&](bool p) -> uint64_t { return __ballot(p) & smask; };
  auto sbcast = [&](uint32_t x, uint32_t k) -> uint32_t { return (uint32_t)__shfl((int)x, (int)(sbase + k)); };
  static_assert(SEG == 8, "a wave's list is shared by its 8 requests");
  // this request's position in the launch order (its count word and its wave's list; the request
  // itself, its row, is ord[position] when the batch was grouped)
  const uint32_t wv = xcd_block(blockIdx.x, gridDim.x, a.ord ? a.xcd_chunk : 0u);
  const uint32_t gid_ = wv * (64 / SEG) + seg;
  const bool valid = gid_ < a.n_req;
  const uint32_t* row = a.grows ? a.grows + (size_t)(valid ? gid_ : 0u) * a.row_words
                                : a.rows + (size_t)(valid ? (a.ord ? a.ord[gid_] : gid_) : 0u) * a.row_words;
  const uint32_t rw = (valid && sl < RW_HDR) ? row[sl] : 0u;
  const uint32_t rw_hi = (SEG < RW_HDR && valid && SEG + sl < RW_HDR) ? row[SEG + sl] : 0u;
  auto hdr = [&](uint32_t k) -> uint32_t { return (SEG >= RW_HDR || k < SEG) ? sbcast(rw, k) : sbcast(rw_hi, k - SEG); };
  const uint32_t* blk = a.heap + hdr(RW_BLK);
  const uint32_t pt = hdr(RW_P), pi = hdr(RW_P + 1), at = hdr(RW_A), ai = hdr(RW_A + 1), rt = hdr(RW_R), ri = hdr(RW_R + 1);
  const uint32_t pn = hdr(RW_PN), rn = hdr(RW_RN), an = hdr(RW_AN);
  const uint32_t p_anc = hdr(RW_PANC), r_anc = hdr(RW_RANC), a_anc = hdr(RW_AANC);
  const uint32_t cm = a.combo_mask;
  const uint32_t nP = (pn >> 31) + ((pn >> AN_KEYS_SHIFT) & AN_KEYS), nA = (an >> 31) + ((an >> AN_KEYS_SHIFT) & AN_KEYS),
                 nR = (rn >> 31) + ((rn >> AN_KEYS_SHIFT) & AN_KEYS);
  uint32_t n_keys = 0;
  if (valid)
    for (uint32_t m = cm; m; m &= m - 1) {
      const uint32_t cb = __builtin_ctz(m);
      n_keys += ((cb & 3) == KC_ENT ? nP : 1u) * (((cb >> 2) & 1) == KC_ENT ? nA : 1u) * ((cb >> 3) == KC_ENT ? nR : 1u);
    }
  // the wave's list: its 8 requests' buckets packed together in found order (each pair tagged with
  // its request's segment), so the wave writes a few whole lines and the candidate pass, which
  // pools the wave's candidates anyway, reads them back in one or two coalesced loads
  uint32_t* pairs = a.scan_list + (size_t)wv * (2 * WAVE_CAP);
  // scope-bitset pass (image.h "scope bitsets"): the principal's list carries the kidx of its owner
  // and key ancestors after its pairs (p_anc == 0: the principal has no entity, no list)
  const bool kbits = BITS && a.scan_filt && a.sbits_words != 0;
  const bool klist = kbits && valid && p_anc != 0;
  const bool stl = !BITS && a.scan_lds != 0;  // UIDs in LDS for the key loop
  const uint32_t* pl = blk + (int32_t)p_anc;  // the principal's list (signed: image.h "ancestor lists")
  const uint32_t nk = (pn >> AN_KEYS_SHIFT) & AN_KEYS;
  constexpr uint32_t LW = 3;  // list elements loaded with a list head
  uint32_t l_lo = 0, l_hd = 0, l_w[LW] = {0, 0, 0};
  // contexts the encoder resolved (image.h RH_SCTX; the row says so): lanes sl < CTXR_SLOTS read
  // them with the key-entity list, and the list slots' heads are not needed
  const bool hres = BITS && klist && (hdr(RW_ASELF) & ASELF_CTXR) != 0;
  uint32_t hcx = CTXR_EMPTY;
  {
    if (hres && sl < CTXR_SLOTS) hcx = blk[RH_SCTX + sl];
    if (stl) {
      const uint32_t n_st = valid ? min(nk, ANC_ST) : 0u;
      for (uint32_t j = sl; j < n_st; j += SEG)
        s_anc[seg][j] = make_uint2(__builtin_nontemporal_load(pl + 2 * j), __builtin_nontemporal_load(pl + 2 * j + 1));
    }
    if (BITS && klist) {
      const uint32_t* kl = pl + 2 * (pn & AN_COUNT);
      for (uint32_t j = sl; j <= min(nk, SCAN_ANC); j += SEG) s_kid[seg][j] = __builtin_nontemporal_load(kl + j);
    }
    // BITS: lane k < popc(l2_lmask) reads the k-th list slot's head and first LW words after it
    // (element count or marker, elements) in the same trip
    if (LOOKUP && BITS && klist && !hres && a.hlists && sl < (uint32_t)__builtin_popcount(a.l2_lmask)) {
      l_lo = row[RW_HDR + 2 * a.n_hot + __popc(a.hlists & ((1u << nth_bit(a.l2_lmask, sl)) - 1u))];
      l_hd = blk[l_lo];
#pragma unroll
      for (uint32_t k = 0; k < LW; k++) l_w[k] = blk[l_lo + 1 + k];  // (past a short list: its block's next words)
    }
    for (uint32_t h = sl; h < min(a.n_hot, SCAN_HOT); h += SEG)
      s_hot[seg][h] = valid ? *reinterpret_cast<const uint2*>(row + RW_HDR + 2 * h) : make_uint2(0u, 0u);
    wave_lds_sync();
  }
  // BITS: the request's presence mask (image.h "presence masks": the encoder's, in the row), which
  // the bitset path tests each listed bucket's mask against; parked in its LDS row's last word, so
  // no register carries it through the key loop
  if constexpr (BITS) {
    const uint32_t pm = (hdr(RW_ASELF) >> ASELF_PRES_SHIFT) & ((1u << ASELF_PRES_SLOTS) - 1u);
    if (sl == 0) s_kid[seg][SCAN_ROW - 1] = pm;
  }
  // level-1 key k of the request: its combo and (principal, action, resource) components
  auto key_at = [&](uint32_t k, uint32_t& cbo, uint2& p, uint2& q, uint2& r) {
    uint32_t j = k, combo = 0;
    bool found = false;
    for (uint32_t m = cm; m; m &= m - 1) {
      const uint32_t cb = __builtin_ctz(m);
      const uint32_t cnt = ((cb & 3) == KC_ENT ? nP : 1u) * (((cb >> 2) & 1) == KC_ENT ? nA : 1u) * ((cb >> 3) == KC_ENT ? nR : 1u);
      if (!found) {
        if (j < cnt) { combo = cb; found = true; }
        else j -= cnt;
      }
    }
    const uint32_t pkc = combo & 3, akc = (combo >> 2) & 1, rkc = combo >> 3;
    const uint32_t np_ = pkc == KC_ENT ? nP : 1u, na_ = akc == KC_ENT ? nA : 1u;
    uint32_t ip = j, ia = 0, ir = 0;
    if (na_ != 1u || (rkc == KC_ENT && nR != 1u)) {
      const uint32_t t2 = j / np_;
      ip = j - t2 * np_; ia = t2 % na_; ir = t2 / na_;
    }
    const uint32_t jp = ip + 1 - (pn >> 31);  // 0: the principal itself, j: ancestor j - 1
    p = (stl && pkc == KC_ENT && jp && jp <= ANC_ST) ? s_anc[seg][jp - 1] : key_comp(pkc, jp, pt, pi, blk, p_anc);
    q = key_comp(akc, ia + 1 - (an >> 31), at, ai, blk, a_anc);
    r = key_comp(rkc, ir + 1 - (rn >> 31), rt, ri, blk, r_anc);
    cbo = combo;
  };
  // Scope-bitset pass (image.h "scope bitsets"). When every used combo's action / resource
  // component is the request's own UID, its one key ancestor, its type or a wildcard (nA, nR <= 1:
  // the k8s SAR shape), each entity-principal combo has a handful of contexts: level 1 and, per hot
  // slot with level-2 keys, the request's value (or each element of its list). The segment's lanes
  // look them up in the context table side by side, then test one bit per (found context,
  // principal key ancestor) pair, all loads of a round in flight at once; only the keys whose bit
  // is set are listed (LIST_EXACT) and probed below, once each, with no level-2 descent. The single
  // keys of the other combos (principal type or wildcard) are listed as combo << 11 and walk both
  // levels as before.
  const uint32_t simple = valid && (!(cm & COMBO_AENT) || nA <= 1u) && (!(cm & COMBO_RENT) || nR <= 1u) && nP < 2048u;
  const uint2 ka1 = (simple && nA == 1u) ? key_comp(KC_ENT, 1u - (an >> 31), at, ai, blk, a_anc) : make_uint2(KW_ANY, KW_ANY);
  const uint2 kr1 = (simple && nR == 1u) ? key_comp(KC_ENT, 1u - (rn >> 31), rt, ri, blk, r_anc) : make_uint2(KW_ANY, KW_ANY);
  auto comb_q = [&](uint32_t cb) { return ((cb >> 2) & 1) == KC_ENT ? ka1 : make_uint2(KW_ANY, KW_ANY); };
  auto comb_r = [&](uint32_t cb) {
    const uint32_t rkc = cb >> 3;
    return rkc == KC_ENT ? kr1 : (rkc == KC_TYPE ? make_uint2(rt, KW_ANY) : make_uint2(KW_ANY, KW_ANY));
  };
  // principal component ip of a combo's keys (0: the UID itself when it is a key entity)
  auto comb_p = [&](uint32_t cb, uint32_t ip) -> uint2 {
    const uint32_t pkc = cb & 3;
    if (pkc != KC_ENT) return key_comp(pkc, 0u, pt, pi, blk, p_anc);
    const uint32_t jp = ip + 1 - (pn >> 31);
    return (stl && jp && jp <= ANC_ST) ? s_anc[seg][jp - 1] : key_comp(KC_ENT, jp, pt, pi, blk, p_anc);
  };
  uint32_t npos = 0;
  bool flt = false;
  if (BITS && __ballot(kbits && klist && simple) != 0) {
    bool on = kbits && klist && simple;
    const uint32_t vm = a.l2_vmask, lm = a.l2_lmask, pe = cm & COMBO_PENT;  // wave-uniform
    const uint32_t nvs = __builtin_popcount(vm), nls = __builtin_popcount(lm), ncb = __builtin_popcount(pe);
    const uint32_t lc = (LOOKUP && on && sl < nls && a.hlists) ? ((l_hd & 0x80000000u) ? 1u : l_hd) : 0u;  // list entries
    uint32_t linc = lc;  // inclusive prefix over the segment's lanes
    for (uint32_t o = 1; o < SEG; o <<= 1) {
      const uint32_t y = (uint32_t)__shfl_up((int)linc, o);
      if (sl >= o) linc += y;
    }
    const uint32_t per = 1u + nvs + sbcast(linc, SEG - 1), nctx = ncb * per;
    on = on && (hres || (LOOKUP && nctx <= CTX_CAP));
    uint32_t nf = 0;  // contexts found (segment-uniform)
    const bool look = LOOKUP && on && !hres;
    if (hres) {  // resolved by the encoder: CTXR_EMPTY after the last
      const bool got = sl < CTXR_SLOTS && hcx != CTXR_EMPTY;
      const uint64_t mk = sballot(got);
      if (got) s_cx[seg][mbcnt64(mk)] = make_uint2(hcx & ((1u << CTXR_ROW) - 1u), hcx >> CTXR_ROW);
      nf = popc64(mk);
    }
    // the contexts, looked up side by side (lane j % SEG takes context j); a found one is kept
    for (uint32_t j0 = 0; __ballot(look && j0 < nctx) != 0; j0 += SEG) {
      const uint32_t j = j0 + sl;
      uint32_t cb = 0, hs = SCTX_L1, v0 = 0, v1 = 0, row_ = KIDX_NONE;
      const uint32_t ci = look ? j / per : 0u, t = look ? j - ci * per : 0u;
      // (the list entry, by shuffles from the lane that read its slot: every lane takes part)
      uint32_t li = 0, lb = 0, llo = 0, lhd = 0, lw = 0;
      for (uint32_t k = 0; k < nls; k++) {
        const uint32_t inc_k = sbcast(linc, k), c_k = sbcast(lc, k);
        const uint32_t u = t - 1 - nvs;
        const bool mine = t > nvs && u < inc_k && u >= inc_k - c_k;
        uint32_t w = 0;
#pragma unroll
        for (uint32_t q = 0; q < LW; q++) {
          const uint32_t wq = sbcast(l_w[q], k);
          if (mine && u - (inc_k - c_k) == q) w = wq;
        }
        const uint32_t lo_k = sbcast(l_lo, k), hd_k = sbcast(l_hd, k);
        if (mine) { li = k; lb = inc_k - c_k; llo = lo_k; lhd = hd_k; lw = w; }
      }
      if (look && j < nctx) {
        cb = nth_bit(pe, ci);
        if (t > 0 && t <= nvs) {
          hs = nth_bit(vm, t - 1);
          const uint2 v = hs < SCAN_HOT ? s_hot[seg][hs] : *reinterpret_cast<const uint2*>(row + RW_HDR + 2 * hs);
          v0 = hot_ok(v) ? v.x : MISSING_W0;
          v1 = hot_ok(v) ? v.y : 0u;
        } else if (t > nvs) {
          hs = nth_bit(lm, li) | BT_CKEY;
          const uint32_t e = t - 1 - nvs - lb;
          if (lhd & 0x80000000u) v0 = lhd == CL_MISSING ? MISSING_W0 : NOTSET_W0;
          else { v0 = e < LW ? lw : blk[llo + 1 + e]; v1 = 1; }
        }
        const uint2 q = comb_q(cb), r = comb_r(cb);
        // (fingerprint, row) pairs only: a fingerprint match is taken without comparing the full
        // key. That stays exact: every key a row lists is probed in the scope table, which compares
        // the whole key, so a row of another context can only add probes that find nothing; and
        // the request's own context (when it exists) matches on its chain, so its bits are never
        // missed. Two matches on one chain (32-bit fingerprints: practically never) enumerate the
        // request's keys instead.
        // the whole 32-byte slot in one trip, compared word for word (exact: a found context's
        // set bits are the request's keys themselves)
        const uint32_t hash = ctx_key(key_pre(cb, q.x, q.y, r.x, r.y), hs, v0, v1), w0c = ctx_w0(cb, hs);
        bool maybe = true;  // the context filter first: most contexts a request names do not exist
        if (a.sbloom) {
          const uint32_t bw = ctx_bloom_words(a.sctx_mask + 1u);
          const uint2 fw = *reinterpret_cast<const uint2*>(a.sbloom + 2 * (size_t)ctx_bloom_at(hash, bw));
          const uint64_t need = ctx_bloom_bits(hash);
          maybe = ((((uint64_t)fw.y << 32) | fw.x) & need) == need;
        }
        for (uint32_t h = hash & a.sctx_mask; maybe; h = (h + 1) & a.sctx_mask) {
          const uint4* slp = reinterpret_cast<const uint4*>(a.sctx + (size_t)h * SCTX_WORDS);
          const uint4 x = slp[0], y = slp[1];
          if (x.x == 0) break;
          if (x.x == w0c && x.y == q.x && x.z == q.y && x.w == r.x && y.x == r.y && y.y == v0 && y.z == v1) {
            row_ = y.w;
            break;
          }
        }
      }
      const bool got = look && j < nctx && row_ != KIDX_NONE;
      const uint64_t mk = sballot(got);
      if (got) s_cx[seg][nf + mbcnt64(mk)] = make_uint2(cb | (hs << 8), row_);
      nf += popc64(mk);
    }
    wave_lds_sync();
    // (found context, key ancestor) pairs: ip 0 .. nP - 1 under each; a set bit lists the key. All
    // SCAN_PB loads of a lane's round in flight at once.
    const uint32_t self = pn >> 31, tot = on ? nf * nP : 0u;
    const uint32_t* kl = pl + 2 * (pn & AN_COUNT);
    // t / nP by a multiply: exact while t * nP < 2^32 (t < CTX_CAP * nP, nP < 2048); nP == 1
    // (whose reciprocal does not fit 32 bits) divides by itself (checked for every nP < 2048 on the
    // host)
    const uint32_t inv = nP > 1 ? 0xFFFFFFFFu / nP + 1u : 0u;
    auto divp = [&](uint32_t t) { return nP > 1 ? __umulhi(t, inv) : t; };
    // a key-entity index past the image's key entities (a batch encoded for another image): the
    // request enumerates every key instead (exact), and is counted so that the batch fails
    bool badk = false;
    for (uint32_t rb = 0; __ballot(rb < tot) != 0; rb += SEG * SCAN_PB) {
      uint2 fw[SCAN_PB];
      uint32_t fb[SCAN_PB];  // the bit's index in its word | combo << 8 (one register per load in flight)
#pragma unroll
      for (uint32_t u = 0; u < SCAN_PB; u++) {
        const uint32_t t = rb + u * SEG + sl;
        fw[u] = make_uint2(0u, 0u);
        fb[u] = 0;
        if (t < tot) {
          const uint32_t j = divp(t), ip = t - j * nP;
          const uint32_t jk = ip + 1 - self;  // kid index: 0 the principal, j key ancestor j - 1
          const uint32_t kid = jk <= SCAN_ANC ? s_kid[seg][jk] : kl[jk];
          const uint2 c = s_cx[seg][j];
          fb[u] = (kid & 31u) | ((c.x & 0xFFu) << 8);
          // the bit's word and the rank of the word's first bit, in one 8-byte load
          if (kid < a.n_kent) fw[u] = *reinterpret_cast<const uint2*>(a.sbits + 2 * ((size_t)c.y * a.sbits_words + (kid >> 5)));
          else badk = badk || kid != KIDX_NONE;
        }
      }
#pragma unroll
      for (uint32_t u = 0; u < SCAN_PB; u++) {
        const uint32_t b = fb[u] & 31u;
        const bool ok = (fw[u].x >> b) & 1u;
        const uint64_t mk = sballot(ok);
        const uint32_t at_ = npos + mbcnt64(mk);
        if (ok && at_ < SCAN_POS_B) s_pos[seg][at_] = LIST_EXACT | ((fb[u] >> 8) << 26) | (fw[u].y + __popc(fw[u].x & ((1u << b) - 1u)));
        npos += popc64(mk);
      }
    }
    if (sballot(badk) != 0) {
      if (on && sl == 0 && a.bad_kidx) atomicAdd(a.bad_kidx, 1u);
      on = false;
    }
    // the other combos' single keys
    for (uint32_t m = cm & ~COMBO_PENT; m; m &= m - 1) {
      if (on && sl == 0 && npos < SCAN_POS_B) s_pos[seg][npos] = __builtin_ctz(m) << 11;
      npos += on ? 1u : 0u;
    }
    wave_lds_sync();
    // a request off the simple shape, with more contexts or listed keys than the lists hold, or
    // more key ancestors than are staged, enumerates every key instead
    flt = on && npos <= SCAN_POS_B;
    if (STATS && sl == 0 && valid) {
      st[11] += flt;
      st[12] += nf;
      st[13] += hres ? 1u : 0u;
      st[14] += npos;
      st[15] += (kbits && klist && simple) ? 1u : 0u;
    }
  }
  const uint32_t n_l1 = flt ? npos : n_keys;
  const uint64_t t1 = STATS ? clock64() : 0;
  if (STATS && valid && sl == 0) { st[0] = 1; st[10] = n_keys; }
  uint32_t kb = 0, hm = 0, h1 = 0, w0 = 0, combo = 0, nb = 0, unused = 0, heads = 0;
  uint32_t wn = 0;        // the wave's list length so far (wave-uniform)
  bool dropped = false;   // a bucket of this lane's request found no room in the wave's list
  uint2 kp = make_uint2(0, 0), ka = kp, kr = kp;
  uint4 blm = make_uint4(0, 0, 0, 0);
  uint32_t csl = 0, ch = 0, cl = 0, ck = 0, cn = 0;
  for (;;) {
    const bool l2 = sballot(hm != 0 || csl != 0 || ck < cn) != 0;
    const bool done = !l2 && kb >= n_l1;
    if (__ballot(!done) == 0) break;
    if (STATS) {
      if (lane == 0) st[5]++;
      if (sl == 0 && !done) { st[7]++; if (l2) st[6]++; }
    }
    uint3 e = make_uint3(0, 0, 0);
    if (!done) {
      if (l2) {
        if (STATS && (hm || csl || ck < cn)) st[3]++;
        if (hm) {
          const uint32_t h = __builtin_ctz(hm);
          hm &= hm - 1;
          const uint2 v = h < SCAN_HOT ? s_hot[seg][h] : *reinterpret_cast<const uint2*>(row + RW_HDR + 2 * h);
          const uint32_t v0 = hot_ok(v) ? v.x : MISSING_W0, v1 = hot_ok(v) ? v.y : 0u;
          const uint32_t h2 = bucket_hash2(h1, h, v0, v1);
          if (l2_bloom_maybe(blm, h2) && (!a.l2filt || filt_maybe(a.bfilt, a.fmask, h2)))
            e = probe(a.btab, a.bmask, h2, w0 | BT_L2 | h, kp, ka, kr, v0, v1, unused, nullptr, nullptr, a.slot_split);
        } else if (csl || ck < cn) {
          uint32_t v0 = 0, v1 = 0;
          bool go = false;
          if (ck >= cn) {
            ch = __builtin_ctz(csl);
            csl &= csl - 1;
            const uint32_t lo = row[RW_HDR + 2 * a.n_hot + __popc(a.hlists & ((1u << ch) - 1u))];
            const uint32_t hd = blk[lo];
            ck = cn = 0;
            if (hd & 0x80000000u) {
              v0 = hd == CL_MISSING ? MISSING_W0 : NOTSET_W0;
              go = true;
            } else {
              cl = lo + 1;
              cn = hd;
            }
          }
          if (!go && ck < cn) {
            v0 = blk[cl + ck];
            v1 = 1;
            ck++;
            go = true;
          }
          if (go) {
            const uint32_t hs = ch | BT_CKEY;
            const uint32_t h2 = bucket_hash2(h1, hs, v0, v1);
            if (l2_bloom_maybe(blm, h2) && (!a.l2filt || filt_maybe(a.bfilt, a.fmask, h2)))
              e = probe(a.btab, a.bmask, h2, w0 | BT_L2 | hs, kp, ka, kr, v0, v1, unused, nullptr, nullptr, a.slot_split);
          }
        }
      } else {
        const uint32_t kk = kb + sl;
        kb += SEG;
        if (kk < n_l1) {
          uint32_t x = 0;
          if (BITS && flt) {
            x = s_pos[seg][kk];
            combo = (x & LIST_EXACT) ? (x >> 26) & 31u : x >> 11;
          } else {
            key_at(kk, combo, kp, ka, kr);
          }
          uint32_t cmv = 0;
          if (BITS && (x & LIST_EXACT)) {  // a key the bitsets found: its bucket at the bit's rank,
                                           // unless it needs an attribute the request lacks
            const uint4 v = *reinterpret_cast<const uint4*>(a.svals + SVAL_WORDS * (size_t)(x & 0x3FFFFFFu));
            const uint32_t pm = s_kid[seg][SCAN_ROW - 1];
            bool keep = (v.z & ~pm) == 0u;
            if (keep && (v.w & EQF_ON)) {  // its policies' equality after the key (image.h "equality filters")
              const uint2 hv = s_hot[seg][(v.w >> EQF_SLOT_SHIFT) & (EQF_SLOTS - 1u)];
              keep = !hot_ok(hv) || eqf_hash(hv.x, hv.y) == (v.w & EQF_HASH);
            }
            e = keep ? make_uint3(v.x, v.y, 0u) : make_uint3(0u, 0u, 0u);
          } else {
            if (BITS && flt) {
              kp = comb_p(combo, 0u);
              ka = comb_q(combo);
              kr = comb_r(combo);
            }
            w0 = BT_USED | (combo << 16);
            h1 = key_hash(combo, kp.x, kp.y, ka.x, ka.y, kr.x, kr.y);
            if (flt || !a.l1filt || filt_maybe(a.bfilt, a.fmask, h1))
              e = probe(a.btab, a.bmask, h1, w0, kp, ka, kr, 0, 0, unused, &blm, &cmv, a.slot_split);
          }
          hm = e.z;
          csl = cmv;
          if (STATS) { st[1]++; if (e.y || hm || csl) st[2]++; }
        }
      }
    }
    if (STATS && l2 && e.y) st[4]++;
    // found buckets go to the wave's list in lane order
    const uint64_t m = __ballot(e.y != 0);
    const uint32_t pos = wn + mbcnt64(m);
    if (e.y) {
      if (pos < WAVE_CAP)
        *reinterpret_cast<uint2*>(pairs + 2 * pos) =
            make_uint2(e.x | (seg << SCAN_SEG_SHIFT), min(e.y, SCAN_COUNT) | (combo << SCAN_COMBO_SHIFT));
      else
        dropped = true;
    }
    wn += popc64(m);
    nb += popc64(m & smask);
    heads += min(e.y, SCAN_COUNT);
  }
  for (uint32_t o = SEG / 2; o > 0; o >>= 1) heads += (uint32_t)__shfl_xor((int)heads, (int)o);  // over the segment
  const bool ovf = sballot(dropped) != 0;
  if (valid && sl == 0) a.scan[gid_] = ovf ? SCAN_OVF : (nb | (heads > a.scan_heavy ? SCAN_HEAVY : 0u));
  if (lane == 0) a.scan_tot[wv] = min(wn, WAVE_CAP);
  if (STATS) {
    const uint64_t t2 = clock64();
    if (lane == 0) { st[8] = (uint32_t)(t1 - t0); st[9] = (uint32_t)(t2 - t1); }
    for (uint32_t i = 0; i < 16; i++) {
      uint32_t x = st[i];
      for (uint32_t o = 32; o > 0; o >>= 1) x += (uint32_t)__shfl_xor((int)x, (int)o);
      if (lane == 0 && x) atomicAdd(a.stats + i, (unsigned long long)x);
    }
  }
}

// SEG lanes evaluate one request; a wave carries 64 / SEG requests whose dependent access chains
// (row -> level-1 probe -> level-2 probe -> head -> atom data) overlap. Collectives (ballot, scan,
// min, broadcast) are segment-local; loops run while any segment of the wave has work.
// STATS: also records, per wave, its work and phase times at a.stats[wave * 16 + i] (profiling
// variant, CEDARGPU_PROBE_STATS=1): [0] requests [1] level-1 keys [2] level-1 buckets found
// [3] level-2 probes [4] level-2 buckets found [5] table slots visited [6] candidate heads
// [7] heads passing the scope re-check [8] atoms evaluated [9] hits [10] stage flushes
// [11] candidate passes; cycles (s_memtime) in [12] row / hot / action loading [13] key probing
// [14] candidate evaluation [15] merge and result writes
// PW: waves per block. Resources are granted per block, so a block's LDS and wave slots return
// only when its slowest wave ends; smaller blocks let fast waves' slots be reused sooner.
// SLIM: the large stage over an image of <= RANK_POL policies (SegLds SLIM words; merge by bitmaps).
template <uint32_t SEG, uint32_t HCAP, uint32_t MINW = 1, bool STATS = false, uint32_t PW = WAVES, bool SPLIT = false,
          bool SLIM = false, uint32_t HOTC = NHOT>
__global__ __launch_bounds__(PW * 64, MINW) void cedar_probe_kernel(KArgs a) {
  const uint64_t t_start = STATS ? clock64() : 0;
  static_assert(!SLIM || (SEG == 64 && HCAP >= 2 * RANK_POL / 32), "SLIM: one-request waves whose hs holds the bitmap");
  using L = SegLds<SEG, HCAP, SLIM, HOTC>;
  static_assert(L::HC <= 4096 && L::XC <= 255, "hit slots are 12-bit sort payloads, error slots 8-bit");
  constexpr uint32_t NS = L::NS;
  __shared__ L wl_all[PW];
  const uint32_t lane = threadIdx.x & 63;
  L& wl = wl_all[threadIdx.x >> 6];
  // (not const: the merge recomputes them, below)
  uint32_t seg = lane / SEG, sl = lane % SEG, sbase = seg * SEG;
  uint64_t smask = SEG == 64 ? ~0ull : (((1ull << SEG) - 1ull) << sbase);
  auto sballot = [&](bool p) -> uint64_t { return __ballot(p) & smask; };
  auto sbcast = [&](uint32_t x, uint32_t k) -> uint32_t { return (uint32_t)__shfl((int)x, (int)(sbase + k)); };
  auto smin = [&](uint32_t x) -> uint32_t {
    for (uint32_t o = SEG / 2; o > 0; o >>= 1) x = min(x, (uint32_t)__shfl_xor((int)x, (int)o));
    return x;
  };
  auto sscan = [&](uint32_t x) -> uint32_t {  // inclusive prefix sum within the segment
    for (uint32_t o = 1; o < SEG; o <<= 1) {
      const uint32_t y = (uint32_t)__shfl_up((int)x, o);
      if (sl >= o) x += y;
    }
    return x;
  };
  const uint32_t blk_w = (PW == 1 && a.ord && !a.req_idx) ? xcd_block(blockIdx.x, gridDim.x, a.xcd_chunk) : blockIdx.x;
  const uint32_t gid = (blk_w * PW + (threadIdx.x >> 6)) * NS + seg;
  const uint32_t n_req = a.n_dev ? min(*a.n_dev, a.n_req) : a.n_req;
  bool valid = gid < n_req;
  // the request's position p in the first pass's launch order (first pass: gid; follow-up: its
  // worklist entry): its scan list and first-pass results are at p, its row at ord[p] when the
  // batch was grouped on the device (grows[p] when the rows were copied into that order)
  const uint32_t p0 = valid ? (a.req_idx ? a.req_idx[gid] : gid) : 0u;
  if (a.req_idx && (p0 & FU_DONE)) valid = false;  // finished by the first pass (its overflow slot)
  if constexpr (SEG == 64 && !STATS) {
    if (!valid) return;  // (a one-request wave with no request: wave-level work only, no block barrier)
  }
  const uint32_t p = valid ? p0 : 0u;
  const uint32_t* row = a.grows ? a.grows + (size_t)p * a.row_words : a.rows + (size_t)(a.ord ? a.ord[p] : p) * a.row_words;
  // FLAT (the SPLIT candidate pass with 8-lane segments): the wave's lanes take candidates from a
  // pool over all of its requests, so each segment's request context and running state live in LDS
  constexpr bool FLAT = SPLIT && SEG == 8;
  static_assert(!SPLIT || FLAT || SEG == 64, "the split pass's list readers: the pooled candidate pass or the large stage");
  static_assert(!FLAT || (NS == 8 && NS * L::EC >= 128), "the pooled candidate pass stages 128 list pairs of its wave");

  // the request row streams through once: non-temporal loads, header broadcast in the segment
  const uint32_t rw = (valid && sl < RW_HDR) ? __builtin_nontemporal_load(row + sl) : 0u;
  // segments narrower than the header hold its upper words in a second register
  const uint32_t rw_hi = (SEG < RW_HDR && valid && SEG + sl < RW_HDR) ? __builtin_nontemporal_load(row + SEG + sl) : 0u;
  // (one-request waves: the header is wave-uniform, read into scalar registers, which keeps the
  // request context out of the large stage's VGPRs)
  auto hdr = [&](uint32_t k) -> uint32_t {
    if constexpr (SEG == 64) return (uint32_t)__builtin_amdgcn_readlane((int)rw, (int)k);
    return (SEG >= RW_HDR || k < SEG) ? sbcast(rw, k) : sbcast(rw_hi, k - SEG);
  };
  // SPLIT: the request's count word, its wave's list total and the list's first 64 (FLAT: 128)
  // pairs, one or two per lane, issued with the row loads (they depend only on the position), so
  // the staging below does not wait for a second trip after the row's. (Past the total the loads
  // read stale pairs of the list's fixed WAVE_CAP region, which the staging ignores.)
  uint32_t scan_nb0 = 0, scan_tot0 = 0;
  uint2 scan_q0 = make_uint2(0u, 0u), scan_q1 = make_uint2(0u, 0u);
  const uint32_t scan_w = FLAT ? gid / NS : p / 8u;  // the wave of the scan that listed the request
  const uint2* scan_l = SPLIT ? reinterpret_cast<const uint2*>(a.scan_list + (size_t)scan_w * (2 * WAVE_CAP)) : nullptr;
  if constexpr (SPLIT) {
    if (valid) scan_nb0 = a.scan[p];
    scan_tot0 = a.scan_tot[scan_w];
    scan_q0 = scan_l[lane];
    if constexpr (FLAT) scan_q1 = scan_l[64 + lane];
  }
  PCtx c;
  c.blk = a.heap + hdr(RW_BLK);
  c.rowb = a.grows ? a.grows : a.rows;
  c.rowo = (valid && a.hlists) ? (uint32_t)(row - c.rowb) + RW_HDR + 2 * a.n_hot : 0xFFFFFFFFu;
  c.lmask = a.hlists;
  c.cpool = a.cpool;
  c.lh = wl.he[seg];  // atoms never address lane scratch (any valid pointer)
  c.gstr_off = a.gstr_off;
  c.gstr_bytes = a.gstr_bytes;
  c.bstr_off = a.bstr_off;
  c.bstr_bytes = a.bstr_bytes;
  c.n_gstr = a.n_gstr;
  c.hotl = wl.hot[seg];
  c.pt = hdr(RW_P); c.pi = hdr(RW_P + 1);
  c.at = hdr(RW_A); c.ai = hdr(RW_A + 1);
  c.rt = hdr(RW_R); c.ri = hdr(RW_R + 1);
  // ancestor counts, and how many of each list (key entities first) the key enumeration takes
  const uint32_t pn = hdr(RW_PN), rn = hdr(RW_RN), an = hdr(RW_AN);
  c.p_anc = hdr(RW_PANC); c.p_nanc = pn & AN_COUNT;
  c.r_anc = hdr(RW_RANC); c.r_nanc = rn & AN_COUNT;
  c.a_anc = hdr(RW_AANC); c.a_nanc = an & AN_COUNT;
  for (uint32_t h = sl; h < a.n_hot; h += SEG)
    wl.hot[seg][h] = valid ? make_uint2(__builtin_nontemporal_load(row + RW_HDR + 2 * h),
                                        __builtin_nontemporal_load(row + RW_HDR + 2 * h + 1))
                           : make_uint2(0u, 0u);
  c.lkb = a.like_base;
  c.lslot = a.lslot;
  if (a.like_base != 0xFFFFFFFFu)  // the like words, as hot entries behind the hot values (the launch
                                   // picks a HOTC that holds them)
    for (uint32_t j = sl; j < 3u * (uint32_t)__popc(a.lslot); j += SEG)
      wl.hot[seg][a.like_base + j] = valid ? make_uint2(__builtin_nontemporal_load(row + a.like_off + 2 * j),
                                                        __builtin_nontemporal_load(row + a.like_off + 2 * j + 1))
                                           : make_uint2(0u, 0u);
  // action masks over the image action table (`==` and `in`), resolved by the encoder
  uint64_t am = 0, as = 0;
  uint32_t aself = 0xFFFFu;
  if (a.amask_ok) {
    am = ((uint64_t)hdr(RW_AM1) << 32) | hdr(RW_AM0);
    const uint32_t self = hdr(RW_ASELF) & ASELF_MASK;
    as = (valid && self < 64u) ? (1ull << self) : 0ull;
    aself = (valid && self < 64u) ? self : 0xFFFFu;
  }
  if constexpr (FLAT) {
    // (every value here was read with the whole wave active: hdr() is a cross-lane read)
    const uint32_t blk_off = (uint32_t)(c.blk - a.heap);
    if (sl == 0) {
      wl.cx[seg][0] = make_uint4(blk_off, c.pt, c.pi, c.at);
      wl.cx[seg][1] = make_uint4(c.ai, c.rt, c.ri, c.p_anc);
      wl.cx[seg][2] = make_uint4(c.r_anc, c.a_anc, c.p_nanc | (c.r_nanc << 16), c.a_nanc | (aself << 16));
      wl.cx[seg][3] = make_uint4(c.rowo, (uint32_t)am, (uint32_t)(am >> 32), 0u);
      wl.sst[seg][0] = 0u;
      wl.sst[seg][1] = 0u;
      wl.sst[seg][2] = a.n_tiers - 1;
      wl.sst[seg][3] = 0u;
      wl.sne[seg] = 0u;
    }
  }
  wave_lds_sync();

  const uint64_t t_load = STATS ? clock64() : 0;
  uint64_t t_cand = 0;
  uint32_t min_tier = a.n_tiers - 1;  // lowest tier with a hit so far (segment-uniform)
  uint32_t nh = 0, nx = 0;            // hits / error details recorded (may exceed capacity)
  uint32_t ne = 0;                    // found buckets staged
  bool general = false;               // needs the stream kernel (structural equality)

  const uint32_t cm = a.combo_mask;
  // entity components: the UID itself when it is a key entity (AN_SELF), then the key entities
  // among its ancestors (listed first); none of the other ancestors can complete a key
  const uint32_t nP = (pn >> 31) + ((pn >> AN_KEYS_SHIFT) & AN_KEYS), nA = (an >> 31) + ((an >> AN_KEYS_SHIFT) & AN_KEYS),
                 nR = (rn >> 31) + ((rn >> AN_KEYS_SHIFT) & AN_KEYS);
  uint32_t n_keys = 0;
  if (valid)
    for (uint32_t m = cm; m; m &= m - 1) {
      const uint32_t cb = __builtin_ctz(m);
      n_keys += ((cb & 3) == KC_ENT ? nP : 1u) * (((cb >> 2) & 1) == KC_ENT ? nA : 1u) * ((cb >> 3) == KC_ENT ? nR : 1u);
    }
  uint32_t st[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};  // STATS only (per lane)
  // runs every segment's staged buckets (ne of them, in LDS): candidate heads, scope re-check,
  // atom graph, hits recorded
  auto flush = [&]() {
    const uint64_t t_c0 = STATS ? clock64() : 0;
    // ---- run every segment's staged buckets ----
    uint32_t carry = 0;
    for (uint32_t b0 = 0; __ballot(b0 < ne); b0 += SEG) {
      const uint32_t b = b0 + sl;
      const uint32_t cnt = b < ne ? wl.u.b.epre[seg][b] : 0u;
      const uint32_t inc = sscan(cnt);
      wave_lds_sync();
      if (b < ne) wl.u.b.epre[seg][b] = carry + inc - cnt;
      carry += sbcast(inc, SEG - 1);
      wave_lds_sync();
    }
    const uint32_t total = carry;
    for (uint32_t base = 0; __ballot(base < total); base += SEG) {
      const uint32_t idx = base + sl;
      bool ok = idx < total;
      uint32_t lo = 0, hi = ne;  // bucket of candidate idx: last b with epre[b] <= idx
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (wl.u.b.epre[seg][mid] <= idx) lo = mid;
        else hi = mid;
      }
      const uint32_t ef = ok ? wl.u.b.efirst[seg][lo] : 0u;
      const uint32_t hidx = ok ? (ef & EF_FIRST) + (idx - wl.u.b.epre[seg][lo]) : 0u;
      const uint32_t bcombo = ef >> EF_COMBO;
      const uint32_t* head = a.bstream + (size_t)hidx * HEAD_WORDS;
      const uint4* d4 = reinterpret_cast<const uint4*>(head);
      const uint4 q0 = d4[0], q1 = d4[1], q2 = d4[2], q3 = d4[3];
      const uint32_t flags = q0.x, kinds = q0.y;
      const uint32_t tier = (flags >> 8) & 0xFF;
      ok = ok && tier <= min_tier;
      const uint32_t pk = kinds & 0xFF, ak = (kinds >> 8) & 0xFF, rk = (kinds >> 16) & 0xFF;
      // scope re-check; an `in` / `is in` entity matched by the bucket key's entity component
      // holds already (the request enumerated that key from its ancestor-or-self list)
      if (ak != SK_ANY) {
        if (a.amask_ok) {
          const uint64_t pm = ((uint64_t)q3.w << 32) | q3.z;
          ok = ok && (((ak == SK_EQ ? as : am) & pm) != 0);
        } else if (ak == SK_EQ) {
          ok = ok && c.at == q1.y && c.ai == q1.z;
        } else if (ak == SK_IN) {
          ok = ok && anc_in(c.blk, c.a_anc, c.a_nanc, c.at, c.ai, q1.y, q1.z);
        } else if (((bcombo >> 2) & 1) != KC_ENT) {
          bool any = false;
          for (uint32_t x = 0; ok && x < q1.y && !any; x++)
            any = anc_in(c.blk, c.a_anc, c.a_nanc, c.at, c.ai, a.cpool[q1.z + 2 * x], a.cpool[q1.z + 2 * x + 1]);
          ok = ok && any;
        }
      }
      if (pk == SK_IS || pk == SK_ISIN) ok = ok && c.pt == q0.z;
      if (pk == SK_EQ) ok = ok && c.pt == q0.w && c.pi == q1.x;
      else if ((pk == SK_IN || pk == SK_ISIN) && (bcombo & 3) != KC_ENT)
        ok = ok && anc_in(c.blk, c.p_anc, c.p_nanc, c.pt, c.pi, q0.w, q1.x);
      if (rk == SK_IS || rk == SK_ISIN) ok = ok && c.rt == q1.w;
      if (rk == SK_EQ) ok = ok && c.rt == q2.x && c.ri == q2.y;
      else if ((rk == SK_IN || rk == SK_ISIN) && (bcombo >> 3) != KC_ENT)
        ok = ok && anc_in(c.blk, c.r_anc, c.r_nanc, c.rt, c.ri, q2.x, q2.y);
      // conditions: this lane's atom graph (first HEAD_ATOMS atoms in the head, the rest and all
      // atom data in the policy's full record at PW_EXT)
      const uint32_t na = (q3.x & 0xFFFFu) / ATOM_WORDS;
      const uint32_t* rec = a.bstream + q3.y;  // PW_EXT (word 13)
      uint32_t pc = ok ? (na ? 0u : AT_SAT) : AT_UNSAT;
      if (STATS) { st[6] += idx < total; st[7] += ok; st[11] += sl == 0; }
      bool err = false;
      Err e{0, 0, 0, 0, 0};
      while (__ballot(pc < na)) {
        if (pc < na) {
          const uint4 at = *reinterpret_cast<const uint4*>((pc < HEAD_ATOMS ? head : rec) + POL_WORDS + ATOM_WORDS * pc);
          const uint32_t rr = eval_atom<false>(c, rec, at.x & 0xFF, (at.x >> 8) & 0xFF, at.y, at.z, at.w, e);
          if (STATS) st[8]++;
          if (rr == 3u) { general = true; pc = AT_UNSAT; }
          else if (rr == 2u) { err = true; pc = AT_UNSAT; }
          else pc = rr ? ((at.x >> 16) & 0xFF) : (at.x >> 24);
        }
      }
      // record hits (segment-local slots): a duplicate class (head word PW_CODE_N, image.h) hits
      // for every member, all sharing the head's error detail
      const bool hit = ok && (err || pc == AT_SAT);
      const uint32_t mlist = q2.w;
      const uint32_t nmem = hit ? (mlist ? ((q3.x >> 16) != 0xFFFFu ? (q3.x >> 16) : a.bstream[mlist]) : 1u) : 0u;  // (head word 12: the class size)
      if (STATS) st[9] += nmem;
      const uint32_t mincl = sscan(nmem);
      const uint64_t xmask = sballot(hit && err);
      const uint32_t xpos = nx + mbcnt64(xmask);
      const uint32_t kind = err ? 2u : (flags & PF_FORBID) ? 1u : 0u;
      const uint32_t hmv = SLIM ? (kind << SLIM_KIND) | (tier << SLIM_TIER) | (min(xpos, 0xFFu) << SLIM_SLOT)
                                : kind | (tier << 8) | (min(xpos, 0xFFu) << 16);
      const uint32_t pos0 = nh + mincl - nmem;
      if (hit && !mlist && pos0 < L::HC) {
        if constexpr (SLIM) {
          wl.hp[seg][pos0] = q2.z | hmv;
        } else {
          wl.hp[seg][pos0] = q2.z;  // PW_CODE: global policy index
          wl.hm[seg][pos0] = hmv;
        }
      }
      // class members. One-request waves (the large stage): every hitting class's list at once.
      // Member m of the segment's classes (in lane order) finds its class lane by a binary search
      // over the lanes' prefix counts, and the lanes load MEMB_U members each per round, all in
      // flight together (one class at a time made its ~230 members from ~30 classes a chain of 30
      // dependent loads: large stage 0.375 -> 0.338 ms, profiles/r03/ab14). 8-lane segments (the
      // candidate pass: a few classes per round) copy one class at a time, coalesced, which costs
      // them fewer registers.
      if constexpr (SEG < 64) {
        for (uint64_t cls = sballot(hit && mlist != 0); __ballot(cls != 0);) {
          const bool act = cls != 0;  // this segment still has a class to copy
          const uint32_t src = act ? (uint32_t)__builtin_ctzll(cls) : lane;
          cls &= act ? cls - 1 : 0ull;
          const uint32_t p0 = (uint32_t)__shfl((int)pos0, (int)src), nm = (uint32_t)__shfl((int)nmem, (int)src);
          const uint32_t mls = (uint32_t)__shfl((int)mlist, (int)src), hv = (uint32_t)__shfl((int)hmv, (int)src);
          const uint32_t ml = act ? mls : 0u;
          if (ml)
            for (uint32_t j = sl; j < nm && p0 + j < L::HC; j += SEG) {
              wl.hp[seg][p0 + j] = a.bstream[ml + 1 + j];
              wl.hm[seg][p0 + j] = hv;
            }
        }
      } else {
        const uint32_t cmc = (hit && mlist) ? nmem : 0u;
        const uint32_t cinc = sscan(cmc), cs = cinc - cmc, ctot = sbcast(cinc, SEG - 1);
        for (uint32_t m0 = 0; __ballot(m0 < ctot); m0 += MEMB_U * SEG) {
          uint32_t dst[MEMB_U], hv[MEMB_U], v[MEMB_U];
#pragma unroll
          for (uint32_t u = 0; u < MEMB_U; u++) {
            const uint32_t m = m0 + u * SEG + sl;
            uint32_t c = 0;  // the largest class lane with cs <= m
            for (uint32_t step = SEG / 2; step > 0; step >>= 1) {
              const uint32_t csn = (uint32_t)__shfl((int)cs, (int)(sbase + c + step));
              if (csn <= m) c += step;
            }
            const uint32_t csc = (uint32_t)__shfl((int)cs, (int)(sbase + c)), pc = (uint32_t)__shfl((int)pos0, (int)(sbase + c));
            const uint32_t mlc = (uint32_t)__shfl((int)mlist, (int)(sbase + c));
            hv[u] = (uint32_t)__shfl((int)hmv, (int)(sbase + c));
            const uint32_t off = m - csc;
            dst[u] = (m < ctot) ? pc + off : L::HC;
            v[u] = dst[u] < L::HC ? a.bstream[mlc + 1 + off] : 0u;
          }
#pragma unroll
          for (uint32_t u = 0; u < MEMB_U; u++)
            if (dst[u] < L::HC) {
              if constexpr (SLIM) {
                wl.hp[seg][dst[u]] = v[u] | hv[u];
              } else {
                wl.hp[seg][dst[u]] = v[u];
                wl.hm[seg][dst[u]] = hv[u];
              }
            }
        }
      }
      if (hit) {
        if (err && xpos < L::XC) {
          wl.he[seg][4 * xpos] = e.code | (e.aux << 8);
          wl.he[seg][4 * xpos + 1] = e.k;
          wl.he[seg][4 * xpos + 2] = e.et;
          wl.he[seg][4 * xpos + 3] = e.ei;
        }
      }
      nh += sbcast(mincl, SEG - 1);
      nx += popc64(xmask);
      min_tier = min(min_tier, smin(hit ? tier : 0xFFu));
    }
    ne = 0;
    if (STATS && sl == 0) st[10]++;
    wave_lds_sync();
    if (STATS) t_cand += clock64() - t_c0;
  };
  // The FLAT candidate pass: the wave's staged candidates (every segment's buckets, prefix-summed)
  // form one pool, 64 a round, so a wave takes as many rounds as its whole pool needs instead of
  // as many as its longest request does (C3: ~1 round where 8-lane segments took ~2). A lane builds
  // its candidate's request context from LDS; hits, error details, the lowest hit tier and the
  // structural flag go to that request's region through LDS atomics (the merge orders hits by policy,
  // so their slots' order does not matter).
  // The staged pairs (n_e of them, FLAT_PAIRS at most) are flat LDS arrays over the wave: ff[i] the
  // bucket word (first head | combo), fp[i] the exclusive prefix of the candidate counts | the
  // pair's segment << FP_SEG; W candidates in all (a request whose hits overflowed staged none).
  auto flush_flat = [&](uint32_t W, uint32_t n_e) {
    const uint64_t t_c0 = STATS ? clock64() : 0;
    const uint32_t* ff = &wl.u.b.efirst[0][0];
    const uint32_t* fp = &wl.u.b.epre[0][0];
    for (uint32_t base = 0; base < W; base += 64) {
      const uint32_t g = base + lane;
      bool ok = g < W;
      uint32_t lo = 0, hi = n_e;  // the pair of candidate g: the last i with prefix[i] <= g (a pair
                                  // of no candidates shares its prefix with the next one, so never)
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if ((fp[mid] & FP_PRE) <= g) lo = mid;
        else hi = mid;
      }
      const uint32_t fw = fp[lo];
      const uint32_t s = ok ? fw >> FP_SEG : 0u;
      const uint32_t ef = ok ? ff[lo] : 0u;
      const uint32_t hidx = ok ? (ef & EF_FIRST) + (g - (fw & FP_PRE)) : 0u;
      const uint32_t bcombo = ef >> EF_COMBO;
      const uint32_t* head = a.bstream + (size_t)(CG_DBG == 4 ? 0u : hidx) * HEAD_WORDS;
      const uint4* d4 = reinterpret_cast<const uint4*>(head);
      const uint4 q0 = d4[0], q1 = d4[1], q2 = d4[2], q3 = d4[3];
      if constexpr (L::ATOMS) {  // the head's first atoms, in flight with its descriptor, parked in LDS
        const uint4 a0 = d4[4], a1 = d4[5];
        wl.at4[0][lane] = a0; wl.at4[1][lane] = a1;
        if (a.park > 2) {
          const uint4 a2 = d4[6], a3 = d4[7];
          wl.at4[2][lane] = a2; wl.at4[3][lane] = a3;
        }
      }
      // the candidate's request (segment s)
      const uint4 x0 = wl.cx[s][0], x1 = wl.cx[s][1], x2 = wl.cx[s][2], x3 = wl.cx[s][3];
      PCtx tc;
      tc.blk = a.heap + x0.x;
      tc.cpool = a.cpool;
      tc.lh = wl.he[s];
      tc.gstr_off = a.gstr_off;
      tc.gstr_bytes = a.gstr_bytes;
      tc.bstr_off = a.bstr_off;
      tc.bstr_bytes = a.bstr_bytes;
      tc.n_gstr = a.n_gstr;
      tc.hotl = wl.hot[s];
      tc.pt = x0.y; tc.pi = x0.z; tc.at = x0.w;
      tc.ai = x1.x; tc.rt = x1.y; tc.ri = x1.z; tc.p_anc = x1.w;
      tc.r_anc = x2.x; tc.a_anc = x2.y; tc.p_nanc = x2.z & 0xFFFFu; tc.r_nanc = x2.z >> 16; tc.a_nanc = x2.w & 0xFFFFu;
      tc.rowb = c.rowb;
      tc.rowo = x3.x;
      tc.lmask = a.hlists;
      tc.lkb = a.like_base;
      tc.lslot = a.lslot;
      const uint64_t tam = ((uint64_t)x3.z << 32) | x3.y;
      const uint32_t tself = x2.w >> 16;
      const uint64_t tas = tself < 64u ? (1ull << tself) : 0ull;
      const uint32_t flags = q0.x, kinds = q0.y;
      const uint32_t tier = (flags >> 8) & 0xFF;
      ok = ok && tier <= wl.sst[s][2];
      const uint32_t pk = kinds & 0xFF, ak = (kinds >> 8) & 0xFF, rk = (kinds >> 16) & 0xFF;
      // scope re-check (as flush)
      if (ak != SK_ANY) {
        if (a.amask_ok) {
          const uint64_t pm = ((uint64_t)q3.w << 32) | q3.z;
          ok = ok && (((ak == SK_EQ ? tas : tam) & pm) != 0);
        } else if (ak == SK_EQ) {
          ok = ok && tc.at == q1.y && tc.ai == q1.z;
        } else if (ak == SK_IN) {
          ok = ok && anc_in(tc.blk, tc.a_anc, tc.a_nanc, tc.at, tc.ai, q1.y, q1.z);
        } else if (((bcombo >> 2) & 1) != KC_ENT) {
          bool any = false;
          for (uint32_t x = 0; ok && x < q1.y && !any; x++)
            any = anc_in(tc.blk, tc.a_anc, tc.a_nanc, tc.at, tc.ai, a.cpool[q1.z + 2 * x], a.cpool[q1.z + 2 * x + 1]);
          ok = ok && any;
        }
      }
      if (pk == SK_IS || pk == SK_ISIN) ok = ok && tc.pt == q0.z;
      if (pk == SK_EQ) ok = ok && tc.pt == q0.w && tc.pi == q1.x;
      else if ((pk == SK_IN || pk == SK_ISIN) && (bcombo & 3) != KC_ENT)
        ok = ok && anc_in(tc.blk, tc.p_anc, tc.p_nanc, tc.pt, tc.pi, q0.w, q1.x);
      if (rk == SK_IS || rk == SK_ISIN) ok = ok && tc.rt == q1.w;
      if (rk == SK_EQ) ok = ok && tc.rt == q2.x && tc.ri == q2.y;
      else if ((rk == SK_IN || rk == SK_ISIN) && (bcombo >> 3) != KC_ENT)
        ok = ok && anc_in(tc.blk, tc.r_anc, tc.r_nanc, tc.rt, tc.ri, q2.x, q2.y);
      const uint32_t na = (q3.x & 0xFFFFu) / ATOM_WORDS;
      const uint32_t* rec = a.bstream + q3.y;  // PW_EXT (word 13)
      uint32_t pc = ok ? (na ? 0u : AT_SAT) : AT_UNSAT;
      if (STATS) { st[6] += g < W; st[7] += ok; st[11] += lane < NS; }
      bool err = false, structural_hit = false;
      Err e{0, 0, 0, 0, 0};
      if (CG_DBG == 1) pc = ok ? AT_SAT : AT_UNSAT;
      while (__ballot(pc < na)) {
        if (STATS && lane == 0) st[10]++;  // (profiling: atom rounds of the wave, in lane 0)
        // (profiling, lane 0: cycles and count of the atom rounds in which some lane evaluates a
        // set atom (RECSET / CONTAINS): st[1], st[2]; of the other rounds: st[3], st[5])
        const uint64_t ta0 = STATS ? clock64() : 0;
        bool set_atom = false;
        if (pc < na) {
          const uint4 at = (L::ATOMS && pc < a.park) ? wl.at4[L::ATOMS ? pc : 0][lane]
                                                          : *reinterpret_cast<const uint4*>((pc < HEAD_ATOMS ? head : rec) + POL_WORDS + ATOM_WORDS * pc);
          if (STATS) set_atom = (at.x & 0xFF) == AK_RECSET || (at.x & 0xFF) == AK_CONTAINS;
          const uint32_t rr = eval_atom<false>(tc, rec, at.x & 0xFF, (at.x >> 8) & 0xFF, at.y, at.z, at.w, e);
          if (STATS) { st[8]++; st[4] += (at.x & 0xFF) == AK_LIKE || (at.x & 0xFF) == AK_LIKEI; }
          if (rr == 3u) { structural_hit = true; pc = AT_UNSAT; }
          else if (rr == 2u) { err = true; pc = AT_UNSAT; }
          else pc = rr ? ((at.x >> 16) & 0xFF) : (at.x >> 24);
        }
        if constexpr (STATS) {
          asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
          const uint32_t dt = (uint32_t)(clock64() - ta0);
          const bool any_set = __ballot(set_atom) != 0;
          if (lane == 0) { if (any_set) { st[1] += dt; st[2]++; } else { st[3] += dt; st[5]++; } }
        }
      }
      const bool hit = ok && (err || pc == AT_SAT);
      const uint32_t mlist = q2.w;
      // a duplicate class that holds (no error) takes one slot under its representative, which the
      // merge reports as an RS_CLASS reason; one that errs records every member with the error
      const bool whole = a.cls && mlist && !err;
      const uint32_t nmem = hit ? ((mlist && !whole) ? ((q3.x >> 16) != 0xFFFFu ? (q3.x >> 16) : a.bstream[mlist]) : 1u) : 0u;  // (head word 12: the class size)
      if (STATS) st[9] += nmem;
      const uint32_t pos0 = hit ? atomicAdd(&wl.sst[s][0], CG_DBG == 2 ? 1u : nmem) : 0u;
      const uint32_t xpos = (hit && err) ? atomicAdd(&wl.sst[s][1], 1u) : 0u;
      const uint32_t kind = err ? 2u : (flags & PF_FORBID) ? 1u : 0u;
      const uint32_t hmv = kind | (tier << 8) | (min(xpos, 0xFFu) << 16) | (whole ? HM_CLASS : 0u);
      if (hit && (!mlist || whole) && pos0 < L::HC) {
        wl.hp[s][pos0] = q2.z;
        wl.hm[s][pos0] = hmv;
      }
      if (CG_DBG != 2 && hit && mlist && !whole) {  // a duplicate class: every member, MEMB_U loads in flight
        for (uint32_t j = 0; j < nmem && pos0 + j < L::HC; j += MEMB_U) {
          uint32_t v[MEMB_U];
#pragma unroll
          for (uint32_t u = 0; u < MEMB_U; u++) v[u] = (j + u < nmem && pos0 + j + u < L::HC) ? a.bstream[mlist + 1 + j + u] : 0u;
#pragma unroll
          for (uint32_t u = 0; u < MEMB_U; u++)
            if (j + u < nmem && pos0 + j + u < L::HC) {
              wl.hp[s][pos0 + j + u] = v[u];
              wl.hm[s][pos0 + j + u] = hmv;
            }
        }
      }
      if (hit && err && xpos < L::XC) {
        wl.he[s][4 * xpos] = e.code | (e.aux << 8);
        wl.he[s][4 * xpos + 1] = e.k;
        wl.he[s][4 * xpos + 2] = e.et;
        wl.he[s][4 * xpos + 3] = e.ei;
      }
      if (hit) atomicMin(&wl.sst[s][2], tier);
      if (structural_hit) atomicOr(&wl.sst[s][3], 1u);
      wave_lds_sync();
    }
    ne = 0;
    if (STATS && sl == 0) st[10]++;
    wave_lds_sync();
    // this request's running state, back in its segment's registers
    nh = wl.sst[seg][0];
    nx = wl.sst[seg][1];
    min_tier = wl.sst[seg][2];
    general = wl.sst[seg][3] != 0u;
    if (STATS) t_cand += clock64() - t_c0;
  };
  uint32_t kb = 0, hm = 0, h1 = 0, w0 = 0, combo = 0;
  uint2 kp = make_uint2(0, 0), ka = kp, kr = kp;
  uint4 blm = make_uint4(0, 0, 0, 0);  // level-2 bloom of this lane's level-1 entry
  // set-membership slots of the entry still to probe (image.h BT_CKEY), the current one's element
  // hash list in the request block and the next element
  uint32_t csl = 0, ch = 0, cl = 0, ck = 0, cn = 0;
  bool probe_loop = !SPLIT;
  if constexpr (SPLIT) {
    // the scan kernel found this request's buckets (cedar_scan_kernel): stage them EC at a time.
    // More buckets than the scan holds: the one-request-per-wave variant probes the index itself,
    // narrower segments hand the request to that variant (the large-stage follow-up).
    const uint32_t nb0 = scan_nb0;
    const bool heavy = nb0 != SCAN_OVF && (nb0 & SCAN_HEAVY);
    const uint32_t nb = nb0 == SCAN_OVF ? SCAN_OVF : (nb0 & ~SCAN_HEAVY);
    if (SEG == 64 && nb == SCAN_OVF) probe_loop = true;
    const bool skip = SEG < 64 && nb != SCAN_OVF && (nb > a.scan_big || heavy) && !a.req_idx;
    if (SEG < 64 && (nb == SCAN_OVF || skip)) nh = L::HC + 1;
    const uint32_t tot = scan_tot0;
    if constexpr (FLAT) {
      // The wave's list, FLAT_PAIRS pairs a round: each pair's candidates counted unless its request
      // is out (skipped, overflowed list, or more hits than this pass holds: the large stage redoes
      // it), prefix-summed over the wave into LDS, then run as one pool (flush_flat).
      if (sl == 0) wl.sst[seg][0] = nh;
      wave_lds_sync();
      uint32_t* ff = &wl.u.b.efirst[0][0];
      uint32_t* fp = &wl.u.b.epre[0][0];
      for (uint32_t b0 = 0; b0 < tot; b0 += FLAT_PAIRS) {
        const uint32_t i0 = b0 + lane, i1 = b0 + 64 + lane;
        const uint2 qa = b0 == 0 ? scan_q0 : (i0 < tot ? scan_l[i0] : make_uint2(0u, 0u));
        const uint2 qb = b0 == 0 ? scan_q1 : (i1 < tot ? scan_l[i1] : make_uint2(0u, 0u));
        const uint32_t sa = (qa.x >> SCAN_SEG_SHIFT) & 7u, sb = (qb.x >> SCAN_SEG_SHIFT) & 7u;
        const uint32_t ca = (i0 < tot && wl.sst[sa][0] <= L::HC) ? (qa.y & SCAN_COUNT) : 0u;
        const uint32_t cb = (i1 < tot && wl.sst[sb][0] <= L::HC) ? (qb.y & SCAN_COUNT) : 0u;
        const uint32_t ia = wave_scan(ca, lane);
        const uint32_t ta = (uint32_t)__builtin_amdgcn_readlane((int)ia, 63);
        const uint32_t ib = wave_scan(cb, lane) + ta;
        ff[lane] = (qa.x & EF_FIRST) | ((qa.y >> SCAN_COMBO_SHIFT) << EF_COMBO);
        ff[64 + lane] = (qb.x & EF_FIRST) | ((qb.y >> SCAN_COMBO_SHIFT) << EF_COMBO);
        fp[lane] = (ia - ca) | (sa << FP_SEG);
        fp[64 + lane] = (ib - cb) | (sb << FP_SEG);
        const uint32_t W = (uint32_t)__builtin_amdgcn_readlane((int)ib, 63);
        wave_lds_sync();
        if constexpr (STATS) {
          // candidate sharing (profiling): the round's candidates, and those of its distinct buckets
          // (a bucket's heads are one range, so the wave's pairs of one bucket share every head),
          // summed over the launch behind the per-wave counters
          const uint32_t n_e = min(FLAT_PAIRS, tot - b0);
          uint32_t tc = 0, dc = 0;
          for (uint32_t u = 0; u < 2; u++) {
            const uint32_t i = u * 64 + lane, c = u ? cb : ca;
            if (i >= n_e || !c) continue;
            bool first = true;
            for (uint32_t j = 0; j < i && first; j++) {
              const uint32_t pj = fp[j] & FP_PRE, pn = j + 1 < n_e ? (fp[j + 1] & FP_PRE) : W;
              first = !(pn > pj && (ff[j] & EF_FIRST) == (ff[i] & EF_FIRST));
            }
            tc += c;
            dc += first ? c : 0u;
          }
          for (uint32_t o = 32; o > 0; o >>= 1) {
            tc += (uint32_t)__shfl_xor((int)tc, (int)o);
            dc += (uint32_t)__shfl_xor((int)dc, (int)o);
          }
          if (lane == 0) {
            atomicAdd(a.stats + (size_t)gridDim.x * 16, (unsigned long long)tc);
            atomicAdd(a.stats + (size_t)gridDim.x * 16 + 1, (unsigned long long)dc);
          }
        }
        flush_flat(W, min(FLAT_PAIRS, tot - b0));
      }
    } else if (nb != SCAN_OVF) {
      // the large stage (one request per wave): this request's pairs of its wave's list, picked by
      // their segment tag 64 at a time and staged in found order
      const uint32_t t = p & 7u;
      for (uint32_t b0 = 0; b0 < tot; b0 += 64) {
        const uint32_t i = b0 + lane;
        const uint2 q = b0 == 0 ? scan_q0 : (i < tot ? scan_l[i] : make_uint2(0u, 0u));
        const bool mine = i < tot && ((q.x >> SCAN_SEG_SHIFT) & 7u) == t;
        const uint64_t m = __ballot(mine);
        if (mine) {
          const uint32_t at = ne + mbcnt64(m);
          wl.u.b.efirst[0][at] = (q.x & EF_FIRST) | ((q.y >> SCAN_COMBO_SHIFT) << EF_COMBO);
          wl.u.b.epre[0][at] = q.y & SCAN_COUNT;
        }
        ne += popc64(m);
        if (ne + 64 > L::EC || b0 + 64 >= tot) {
          wave_lds_sync();
          if (ne) flush();
        }
      }
    }
  }
  if (probe_loop)
  for (;;) {
    const bool l2 = sballot(hm != 0 || csl != 0 || ck < cn) != 0;
    const bool done = !l2 && kb >= n_keys;
    const bool all_done = __ballot(!done) == 0;
    if (!all_done) {
      uint3 e = make_uint3(0, 0, 0);
      if (!done) {
        if (l2) {
          if (hm) {
            const uint32_t h = __builtin_ctz(hm);
            hm &= hm - 1;
            const uint2 v = wl.hot[seg][h];
            const uint32_t v0 = hot_ok(v) ? v.x : MISSING_W0, v1 = hot_ok(v) ? v.y : 0u;
            const uint32_t h2 = bucket_hash2(h1, h, v0, v1);
            if (l2_bloom_maybe(blm, h2)) {
              if (!a.l2filt || filt_maybe(a.bfilt, a.fmask, h2))
                e = probe<STATS>(a.btab, a.bmask, h2, w0 | BT_L2 | h, kp, ka, kr, v0, v1, st[5], nullptr, nullptr, a.slot_split);
              if (STATS) { st[3]++; st[4] += e.y != 0; }
            }
          } else if (csl || ck < cn) {
            uint32_t v0 = 0, v1 = 0;
            bool go = false;
            if (ck >= cn) {  // the next set-membership slot: its list header
              ch = __builtin_ctz(csl);
              csl &= csl - 1;
              const uint32_t lo = row[RW_HDR + 2 * a.n_hot + __popc(a.hlists & ((1u << ch) - 1u))];
              const uint32_t hd = c.blk[lo];
              ck = cn = 0;
              if (hd & 0x80000000u) {
                v0 = hd == CL_MISSING ? MISSING_W0 : NOTSET_W0;
                go = true;
              } else {
                cl = lo + 1;
                cn = hd;
              }
            }
            if (!go && ck < cn) {
              v0 = c.blk[cl + ck];
              v1 = 1;
              ck++;
              go = true;
            }
            if (go) {
              const uint32_t hs = ch | BT_CKEY;
              const uint32_t h2 = bucket_hash2(h1, hs, v0, v1);
              if (l2_bloom_maybe(blm, h2)) {
                if (!a.l2filt || filt_maybe(a.bfilt, a.fmask, h2))
                  e = probe<STATS>(a.btab, a.bmask, h2, w0 | BT_L2 | hs, kp, ka, kr, v0, v1, st[5], nullptr, nullptr, a.slot_split);
                if (STATS) { st[3]++; st[4] += e.y != 0; }
              }
            }
          }
        } else {
          // (a variant where each lane took its own next level-1 key while others probed level 2
          // was 15 % slower: the two paths then run divergently in every step; profiles/r02/ab_mix)
          const uint32_t k = kb + sl;
          kb += SEG;
          uint32_t j = k;
          bool found = false;
          for (uint32_t m = cm; m; m &= m - 1) {
            const uint32_t cb = __builtin_ctz(m);
            const uint32_t cnt = ((cb & 3) == KC_ENT ? nP : 1u) * (((cb >> 2) & 1) == KC_ENT ? nA : 1u) * ((cb >> 3) == KC_ENT ? nR : 1u);
            if (!found) {
              if (j < cnt) { combo = cb; found = true; }
              else j -= cnt;
            }
          }
          if (k < n_keys) {
            const uint32_t pkc = combo & 3, akc = (combo >> 2) & 1, rkc = combo >> 3;
            const uint32_t np_ = pkc == KC_ENT ? nP : 1u, na_ = akc == KC_ENT ? nA : 1u;
            uint32_t ip = j, ia = 0, ir = 0;
            if (na_ != 1u || (rkc == KC_ENT && nR != 1u)) {  // only the principal varies: no division
              const uint32_t t2 = j / np_;
              ip = j - t2 * np_; ia = t2 % na_; ir = t2 / na_;
            }
            kp = key_comp(pkc, ip + 1 - (pn >> 31), c.pt, c.pi, c.blk, c.p_anc);
            ka = key_comp(akc, ia + 1 - (an >> 31), c.at, c.ai, c.blk, c.a_anc);
            kr = key_comp(rkc, ir + 1 - (rn >> 31), c.rt, c.ri, c.blk, c.r_anc);
            w0 = BT_USED | (combo << 16);
            h1 = key_hash(combo, kp.x, kp.y, ka.x, ka.y, kr.x, kr.y);
            uint32_t cmv = 0;
            if (!a.l1filt || filt_maybe(a.bfilt, a.fmask, h1))
              e = probe<STATS>(a.btab, a.bmask, h1, w0, kp, ka, kr, 0, 0, st[5], &blm, &cmv, a.slot_split);
            hm = e.z;
            csl = cmv;
            if (STATS) st[1]++;
            if (STATS) st[2] += e.y != 0;
          }
        }
      }
      // stage this lane's found bucket in its segment
      const uint64_t m = sballot(e.y != 0);
      if (e.y) {
        const uint32_t pos = ne + mbcnt64(m);
        wl.u.b.efirst[seg][pos] = e.x | (combo << EF_COMBO);
        wl.u.b.epre[seg][pos] = e.y;
      }
      ne += popc64(m);
      wave_lds_sync();
    }
    if (all_done || __ballot(ne + SEG > L::EC)) flush();
    if (all_done) break;
  }
  const uint64_t t_loop = STATS ? clock64() : 0;
  // ---- merge: deciding tier, duplicates, policy order ----
  // The lane's indices and result slot are recomputed here from an opaque lane id (and the request
  // order reloaded) instead of living across the candidate loop: kept live, they were the
  // candidate pass's register spills, whose scratch stores were ~0.2 GB of writes per 1M step.
  uint32_t lane_m = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  asm volatile("" : "+v"(lane_m));
  seg = lane_m / SEG; sl = lane_m % SEG; sbase = seg * SEG;
  smask = SEG == 64 ? ~0ull : (((1ull << SEG) - 1ull) << sbase);
  const uint32_t gid_m = (((PW == 1 && a.ord && !a.req_idx) ? xcd_block(blockIdx.x, gridDim.x, a.xcd_chunk) : blockIdx.x) * PW + (threadIdx.x >> 6)) * NS + seg;
  valid = gid_m < n_req && !(a.req_idx && (a.req_idx[gid_m] & FU_DONE));
  // result slot (FLAT: the request index parked in its context row, an LDS read instead of a
  // dependent reload of the order)
  // result slot: the request's position (first pass) or its worklist entry (follow-up)
  const uint32_t wo = valid ? gid_m : 0u;
  const uint32_t t = min_tier;
  const bool structural = sballot(general) != 0;
  const bool undecided = (CG_DBG == 3 && FLAT) ? false : (nh > L::HC || nx > L::XC || structural);
  if constexpr (CG_DBG == 3 && FLAT) {  // (diagnostic: the merge skipped)
    if (valid && sl == 0) {
      a.res[2 * (size_t)wo] = DEC_DENY | (t << 8) | (RF_VALID << 16);
      a.res[2 * (size_t)wo + 1] = 0;
    }
    return;
  }
  if (valid && undecided && sl == 0) {
    const uint32_t why = (structural || L::HC >= 1024) ? RF_GENERAL : RF_BIG;
    a.res[2 * (size_t)wo] = DEC_DENY | (t << 8) | ((RF_VALID | RF_OVERFLOW | why) << 16);
    a.res[2 * (size_t)wo + 1] = min(nh, 0xFFFFu) | (min(nh, 0xFFFFu) << 16);  // capacity hint

  }
  uint32_t nf = 0, np = 0, nerr = 0;  // distinct deciding forbids / permits / errors
  uint32_t oslot = 0xFFFFFFFFu;       // the overflow slot this request's result went to (SLIM)
  if constexpr (SLIM) {
    // Merge by bitmaps over policy indices (wl.u.hs: the bitmap, then prefix popcounts per word):
    // the deciding tier's forbids are marked first; when none, its permits. Every such hit then
    // stores its policy at its rank among the marked ones (a duplicate stores the same index to the
    // same place), and the errors the same way: the reasons come out in policy order with no sort,
    // no hm words and no sort keys in LDS.
    if (!undecided) {
      uint32_t* bm = wl.u.hs[0];
      uint32_t* pre = wl.u.hs[0] + RANK_POL / 32;
      const uint32_t W = (a.n_pol + 31) >> 5;
      const uint32_t per = (W + 63) / 64, w0 = min(W, lane_m * per), w1 = min(W, w0 + per);
      auto sel = [&](uint32_t x, uint32_t kind) {
        return ((x >> SLIM_TIER) & 0xFFu) == t && ((x >> SLIM_KIND) & 3u) == kind;
      };
      auto mark = [&](uint32_t kind) -> uint32_t {  // bitmap and prefix counts; the distinct count
        for (uint32_t w = lane_m; w < W; w += 64) bm[w] = 0u;
        wave_lds_sync();
        for (uint32_t i = lane_m; i < nh; i += 64) {
          const uint32_t x = wl.hp[0][i];
          if (sel(x, kind)) atomicOr(&bm[(x & SLIM_POL) >> 5], 1u << (x & 31u));
        }
        wave_lds_sync();
        uint32_t cnt = 0;
        for (uint32_t w = w0; w < w1; w++) cnt += __popc(bm[w]);
        uint32_t inc = cnt;
        for (uint32_t o = 1; o < 64; o <<= 1) {
          const uint32_t y = (uint32_t)__shfl_up((int)inc, o);
          if (lane_m >= o) inc += y;
        }
        uint32_t run = inc - cnt;
        for (uint32_t w = w0; w < w1; w++) {
          pre[w] = run;
          run += __popc(bm[w]);
        }
        wave_lds_sync();
        return (uint32_t)__shfl((int)inc, 63);
      };
      auto rank = [&](uint32_t p) { return pre[p >> 5] + __popc(bm[p >> 5] & ((1u << (p & 31u)) - 1u)); };
      nf = mark(1u);
      if (!nf) np = mark(0u);
      const uint32_t kd = nf ? 1u : 0u;
      // a deciding list longer than the request's slot: an overflow slot when the launch has them
      if (a.ovf_cnt && valid && (nf ? nf : np) > a.capr) {
        uint32_t o = 0;
        if (lane_m == 0) o = atomicAdd(a.ovf_cnt, 1u);
        o = (uint32_t)__shfl((int)o, 0);
        oslot = o < a.ovf_cap ? o : 0xFFFFFFFFu;
      }
      uint32_t* rdst = oslot != 0xFFFFFFFFu ? a.ovf_rf + (size_t)oslot * a.ovf_capr : a.reasons_f + (size_t)wo * a.capr;
      const uint32_t rcap = oslot != 0xFFFFFFFFu ? a.ovf_capr : a.capr;
      bool anyerr = false;
      for (uint32_t i = lane_m; i < nh; i += 64) {
        const uint32_t x = wl.hp[0][i];
        anyerr = anyerr || sel(x, 2u);
        if (sel(x, kd)) {
          const uint32_t p = x & SLIM_POL, rk = rank(p);
          if (rk < rcap) __builtin_nontemporal_store(p, rdst + rk);
        }
      }
      if (__ballot(anyerr)) {
        wave_lds_sync();
        nerr = mark(2u);
        const uint32_t ecap = oslot != 0xFFFFFFFFu ? a.ovf_cape : a.cape;
        uint32_t* edst = oslot != 0xFFFFFFFFu ? a.ovf_er + (size_t)oslot * a.ovf_cape * ERR_WORDS : a.errs + (size_t)wo * a.cape * ERR_WORDS;
        for (uint32_t i = lane_m; i < nh; i += 64) {
          const uint32_t x = wl.hp[0][i];
          if (!sel(x, 2u)) continue;
          const uint32_t p = x & SLIM_POL, rk = rank(p), xs = x >> SLIM_SLOT;
          if (rk < ecap) {
            uint32_t* er = edst + (size_t)rk * ERR_WORDS;
            er[0] = p; er[1] = wl.he[0][4 * xs]; er[2] = wl.he[0][4 * xs + 1]; er[3] = wl.he[0][4 * xs + 2];
            er[4] = wl.he[0][4 * xs + 3]; er[5] = 0;
          }
        }
      }
    }
  } else {
    uint32_t nhm = undecided ? 0u : nh;  // this segment's hits to merge (after a rank pass: unique ones)
    // One-request waves with many hits over an image of <= RANK_POL policies: a rank pass instead of
    // the sort. A bitmap over policy indices (hs[0, 512)) takes every hit, prefix popcounts per word
    // (hs[512, 1024)) give each hit its rank among the distinct policies, and the hits scatter to
    // their ranks: five LDS passes instead of ~36 bitonic stages over 256-1024 keys (the large
    // stage's merge was half its time: ~230 hits per request on C3, profiles/r03/ab14).
    bool ranked = false;
    if constexpr (SEG == 64 && HCAP >= 1024) {
      if (nhm > 128 && a.n_pol <= RANK_POL) {
        ranked = true;
        uint32_t* bm = wl.u.hs[0];
        uint32_t* pre = wl.u.hs[0] + RANK_POL / 32;
        const uint32_t W = (a.n_pol + 31) >> 5;
        for (uint32_t w = lane_m; w < W; w += 64) bm[w] = 0u;
        wave_lds_sync();
        for (uint32_t i = lane_m; i < nhm; i += 64) {
          const uint32_t p = wl.hp[0][i];
          atomicOr(&bm[p >> 5], 1u << (p & 31));
        }
        wave_lds_sync();
        const uint32_t per = (W + 63) / 64, w0 = min(W, lane_m * per), w1 = min(W, w0 + per);
        uint32_t cnt = 0;
        for (uint32_t w = w0; w < w1; w++) cnt += __popc(bm[w]);
        uint32_t inc = cnt;
        for (uint32_t o = 1; o < 64; o <<= 1) {
          const uint32_t y = (uint32_t)__shfl_up((int)inc, o);
          if (lane_m >= o) inc += y;
        }
        uint32_t run = inc - cnt;
        for (uint32_t w = w0; w < w1; w++) {
          pre[w] = run;
          run += __popc(bm[w]);
        }
        const uint32_t uniq = (uint32_t)__shfl((int)inc, 63);
        wave_lds_sync();
        for (uint32_t i = lane_m; i < nhm; i += 64) {  // (the hit's policy keeps its place in hp)
          const uint32_t p = wl.hp[0][i];
          const uint32_t r = pre[p >> 5] + __popc(bm[p >> 5] & ((1u << (p & 31)) - 1u));
          wl.hp[0][i] = (r << 16) | p;
        }
        wave_lds_sync();
        for (uint32_t i = lane_m; i < nhm; i += 64) {  // duplicates write the same rank: either is kept
          const uint32_t x = wl.hp[0][i];
          wl.u.hs[0][x >> 16] = ((x & 0xFFFFu) << 12) | i;
        }
        wave_lds_sync();
        nhm = uniq;
      }
    }
    // bitonic sort of (policy index << 12 | slot) over the wave's largest power of two >= nh
    uint32_t mloc = 2;
    while (!ranked && mloc < nhm) mloc <<= 1;
    uint32_t m = ranked ? 0u : mloc;
    // (a bpermute on lane_m: __shfl_xor's own lane id is the prologue's, which then stays live)
    for (uint32_t o = 32; o > 0; o >>= 1) m = max(m, (uint32_t)__builtin_amdgcn_ds_bpermute((int)((lane_m ^ o) << 2), (int)m));
    // Small merges (every segment of the wave <= a.cnt_rank hits): each hit's rank is the number of
    // the segment's keys below its own, every compare's LDS read in flight at once, instead of the
    // bitonic network's log^2 dependent stages (keys are unique: the slot is in the low bits).
    const bool counted = !ranked && m <= a.cnt_rank;
    if (counted) {
      for (uint32_t i = sl; i < nhm; i += SEG) {
        const uint32_t ki = (wl.hp[seg][i] << 12) | i;
        uint32_t rk = 0;
        for (uint32_t j = 0; j < nhm; j += 4) {
          const uint4 h4 = *reinterpret_cast<const uint4*>(&wl.hp[seg][j]);
          rk += (((h4.x << 12) | j) < ki) ? 1u : 0u;
          rk += (j + 1 < nhm && ((h4.y << 12) | (j + 1)) < ki) ? 1u : 0u;
          rk += (j + 2 < nhm && ((h4.z << 12) | (j + 2)) < ki) ? 1u : 0u;
          rk += (j + 3 < nhm && ((h4.w << 12) | (j + 3)) < ki) ? 1u : 0u;
        }
        wl.u.hs[seg][rk] = ki;
      }
      wave_lds_sync();
    }
    for (uint32_t i = sl; !ranked && !counted && i < m; i += SEG) wl.u.hs[seg][i] = i < nhm ? ((wl.hp[seg][i] << 12) | i) : 0xFFFFFFFFu;
    wave_lds_sync();
    for (uint32_t k = 2; !ranked && !counted && k <= m; k <<= 1) {
      for (uint32_t jj = k >> 1; jj > 0; jj >>= 1) {
        for (uint32_t i0 = 0; i0 < (m >> 1); i0 += SEG) {
          const uint32_t q = i0 + sl;  // compare-exchange pair q
          if (q < (m >> 1)) {
            const uint32_t lo = ((q & ~(jj - 1u)) << 1) | (q & (jj - 1u)), hi = lo + jj;  // (jj: a power of two)
            const uint32_t x = wl.u.hs[seg][lo], y = wl.u.hs[seg][hi];
            const bool up = (lo & k) == 0;
            if ((x > y) == up) { wl.u.hs[seg][lo] = y; wl.u.hs[seg][hi] = x; }
          }
        }
        wave_lds_sync();
      }
    }
    // deciding-tier hits, duplicates (adjacent after the sort) dropped; ranks by prefix counts.
    // Only the deciding list is written, into reasons_f (the host passes reasons_p == reasons_f):
    // a first sweep learns whether any forbid decides.
    auto deciding = [&](uint32_t i, uint32_t& pj, uint32_t& mj) {
      const bool have = i < nhm;
      const uint32_t key = have ? wl.u.hs[seg][i] : 0xFFFFFFFFu;
      pj = key >> 12;
      mj = have ? wl.hm[seg][key & 0xFFF] : 0u;
      return have && ((mj >> 8) & 0xFF) == t && (i == 0 || (wl.u.hs[seg][i - 1] >> 12) != pj);
    };
    bool deny = false;
    uint32_t tf = 0, tp = 0, te = 0;  // the deciding lists' lengths
    for (uint32_t c0 = 0; __ballot(c0 < nhm); c0 += SEG) {
      uint32_t pj, mj;
      const bool el = deciding(c0 + sl, pj, mj);
      tf += popc64(sballot(el && (mj & 0xFF) == 1));
      tp += popc64(sballot(el && (mj & 0xFF) == 0));
      te += popc64(sballot(el && (mj & 0xFF) == 2));
    }
    deny = tf != 0;
    // A list longer than the request's capacity (at most 64 reasons and 8 errors here): its whole
    // result goes to an overflow slot of the long-list follow-up's worklist (KArgs::ovf_*, taken in
    // the first pass of a large batch), flagged done, so that follow-up has nothing left to run
    // (only a result the slot holds whole: duplicate classes record a hit per member, so a request
    // decided with 8 error details may list 50 errors; such a one keeps RF_OVERFLOW and the re-runs)
    if (a.ovf_cnt && valid && ((deny ? tf : tp) > a.capr || te > a.cape) && (deny ? tf : tp) <= a.ovf_capr && te <= a.ovf_cape) {
      uint32_t o = 0;
      if (sl == 0) o = atomicAdd(a.ovf_cnt, 1u);
      o = sbcast(o, 0);
      oslot = o < a.ovf_cap ? o : 0xFFFFFFFFu;
    }
    const uint32_t rcap = oslot != 0xFFFFFFFFu ? a.ovf_capr : a.capr, ecap = oslot != 0xFFFFFFFFu ? a.ovf_cape : a.cape;
    uint32_t* rdst = oslot != 0xFFFFFFFFu ? a.ovf_rf + (size_t)oslot * a.ovf_capr : a.reasons_f + (size_t)wo * a.capr;
    uint32_t* edst = oslot != 0xFFFFFFFFu ? a.ovf_er + (size_t)oslot * a.ovf_cape * ERR_WORDS : a.errs + (size_t)wo * a.cape * ERR_WORDS;
    for (uint32_t c0 = 0; __ballot(c0 < nhm); c0 += SEG) {
      uint32_t pj, mj;
      const bool el = deciding(c0 + sl, pj, mj);
      const uint32_t kind = mj & 0xFF;
      const uint64_t bf = sballot(el && kind == 1), bp = sballot(el && kind == 0), be = sballot(el && kind == 2);
      const uint32_t rf = nf + mbcnt64(bf), rp = np + mbcnt64(bp), re = nerr + mbcnt64(be);
      const uint32_t pw = pj | ((mj & HM_CLASS) ? RS_CLASS : 0u);
      if (el && deny && kind == 1 && rf < rcap) __builtin_nontemporal_store(pw, rdst + rf);
      if (el && !deny && kind == 0 && rp < rcap) __builtin_nontemporal_store(pw, rdst + rp);
      if (el && kind == 2 && re < ecap) {
        const uint32_t xs = mj >> 16;
        uint32_t* er = edst + (size_t)re * ERR_WORDS;
        er[0] = pj; er[1] = wl.he[seg][4 * xs]; er[2] = wl.he[seg][4 * xs + 1]; er[3] = wl.he[seg][4 * xs + 2];
        er[4] = wl.he[seg][4 * xs + 3]; er[5] = 0;
      }
      nf += popc64(bf);
      np += popc64(bp);
      nerr += popc64(be);
    }
  }
  if (valid && !undecided && sl == 0) {
    const uint32_t dec = nf ? DEC_DENY : (np ? DEC_ALLOW : DEC_DENY);
    const uint32_t nr = nf ? nf : np;
    uint32_t fl = RF_VALID | (nf ? RF_FORBID : 0u);
    if (oslot != 0xFFFFFFFFu) {  // the whole result in the overflow slot; the request's own says so
      const uint32_t fo = fl | ((nr > a.ovf_capr || nerr > a.ovf_cape) ? RF_OVERFLOW : 0u);
      a.ovf_ids[oslot] = wo | (SLIM ? 0u : FU_DONE);
      a.ovf_res[2 * (size_t)oslot] = dec | (t << 8) | (fo << 16);
      a.ovf_res[2 * (size_t)oslot + 1] = min(nr, 0xFFFFu) | (min(nerr, 0xFFFFu) << 16);
    }
    // (a large batch's slot holds the final result: the request's own then carries no RF_OVERFLOW,
    // which would list it for the follow-up again)
    if ((nr > a.capr || nerr > a.cape) && (SLIM || oslot == 0xFFFFFFFFu)) fl |= RF_OVERFLOW;
    a.res[2 * (size_t)wo] = dec | (t << 8) | (fl << 16);
    a.res[2 * (size_t)wo + 1] = min(nr, 0xFFFFu) | (min(nerr, 0xFFFFu) << 16);
  }
  if (STATS) {
    if (valid && sl == 0) st[0] = 1;
    const uint64_t t_end = clock64();
    unsigned long long* w = a.stats + ((size_t)blockIdx.x * PW + (threadIdx.x >> 6)) * 16;
    for (uint32_t i = 0; i < 12; i++) {
      uint32_t x = valid ? st[i] : 0u;
      for (uint32_t o = 32; o > 0; o >>= 1) x += (uint32_t)__shfl_xor((int)x, (int)o);
      if (lane_m == 0) w[i] = x;
    }
    if (lane_m == 0) {
      w[12] = t_load - t_start;
      w[13] = (t_loop - t_load) - t_cand;
      w[14] = t_cand;
      w[15] = t_end - t_loop;
    }
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

// scalars and array pointers of a device image whose region sits at `base` (blob offset `origin`)
static void image_fields(const Image& img, int device, void* base, uint64_t origin, DevImage& d) {
  d.device = device;
  d.base = base;
  d.origin = origin;
  d.region = img.dev_end - img.dev_begin;
  d.bytes = d.region;
  auto at = [&](uint32_t k) { return (uint8_t*)base + (img.dev_off[k] - origin); };
  d.pstream = (uint32_t*)at(DS_PSTREAM); d.tier_cend = (uint32_t*)at(DS_TIER_CEND); d.chunks = (uint32_t*)at(DS_CHUNKS);
  d.cpool = (uint32_t*)at(DS_CPOOL); d.gstr_off = (uint32_t*)at(DS_GSTR_OFF); d.hot = (uint32_t*)at(DS_HOT);
  d.act = (uint32_t*)at(DS_ACT); d.btab = (uint32_t*)at(DS_BTAB); d.bfilt = (uint32_t*)at(DS_BFILT);
  d.bstream = (uint32_t*)at(DS_BSTREAM); d.srows = (uint32_t*)at(DS_SROWS); d.shash = (uint32_t*)at(DS_SHASH);
  d.sctx = (uint32_t*)at(DS_SCTX); d.sbits = (uint32_t*)at(DS_SBITS); d.svals = (uint32_t*)at(DS_SVALS);
  d.sbloom = (uint32_t*)at(DS_SBLOOM);
  d.sctx_mask = (uint32_t)(img.dev_len[DS_SCTX] / 4 / SCTX_WORDS) - 1;
  d.sbits_words = img.sbits_words;
  d.n_kent = (uint32_t)img.key_ents.size();
  d.l2_vmask = img.l2_vmask;
  d.l2_lmask = img.l2_lmask;
  d.gstr_bytes = at(DS_GSTR_BYTES);
  d.n_static = img.n_static();
  d.lane_need = img.lane_need;
  d.cslot_mask = img.list_mask();
  d.lslot_mask = img.lslot_mask;
  d.like_off = img.like_off();
  d.cls_compact = img.cls_off.empty() ? 0u : 1u;
  d.smask = (uint32_t)(img.shash.size() / SH_WORDS) - 1;
  d.bmask = img.btab_slots - 1;
  d.fmask = (uint32_t)(img.dev_len[DS_BFILT] / 8) - 1;
  d.indexed = img.indexed;
  d.combo_mask = img.combo_mask;
  d.n_act = (uint32_t)img.act.size() / 2;
  d.has_bytecode = img.n_atomic < img.n_pol() ? 1u : 0u;
  d.amask_ok = img.amask_ok;
  d.n_pol = img.n_pol();
  d.n_tiers = img.n_tiers();
  d.n_gstr = img.n_gstr();
  d.n_hot = (uint32_t)img.hot.size() / HOT_WORDS;
}

// One thread per scope-index entry: claims the first free slot of its key's linear-probe chain
// (compare-and-swap of the slot's first word, never 0 in a used slot) and writes the rest. Keys
// are distinct, so any insertion order yields a table every probe (probe()) resolves alike.
// Two launches: level-1 entries (every request probes them) first, so that they head their probe
// chains and a level-2 entry never lengthens a level-1 probe (as the host-built tables had it;
// one mixed launch cost the C3 scan ~5 %, profiles/r03/bis).
__global__ void __launch_bounds__(256) cedar_btab_build(const uint32_t* __restrict__ ent, uint32_t n,
                                                        uint32_t* __restrict__ tab, uint32_t mask, uint32_t level2) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint4* e = reinterpret_cast<const uint4*>(ent + (size_t)i * BT_WORDS);
  const uint4 a = e[0], b = e[1], c = e[2], d = e[3];
  if (a.x == 0) return;  // the placeholder of an image without entries
  if (((a.x & BT_L2) != 0) != (level2 != 0)) return;
  const uint32_t combo = (a.x & ~BT_USED) >> 16;
  uint32_t h = key_hash(combo, a.y, a.z, a.w, b.x, b.y, b.z);
  if (a.x & BT_L2) h = bucket_hash2(h, a.x & 0xFFu & ~BT_L2, b.w, c.x);
  for (h &= mask;; h = (h + 1) & mask)
    if (atomicCAS(tab + (size_t)h * BT_WORDS, 0u, a.x) == 0u) break;
  uint4* t = reinterpret_cast<uint4*>(tab + (size_t)h * BT_WORDS);
  t[0] = make_uint4(a.x, a.y, a.z, a.w);
  t[1] = b;
  t[2] = c;
  t[3] = d;
}

// Builds the image's slot table from its entry list (d.btab points at the list in the region).
static int build_btab(const Image& img, DevImage& d) {
  const size_t bytes = (size_t)img.btab_slots * BT_WORDS * 4;
  const uint32_t n = (uint32_t)(img.dev_len[DS_BTAB] / 4 / BT_WORDS);
  hipStream_t s;
  HIPCHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreate");
  hipError_t e = hipMalloc(&d.btab_mem, bytes);
  if (e == hipSuccess) e = hipMemsetAsync(d.btab_mem, 0, bytes, s);
  if (e == hipSuccess) {
    for (uint32_t l2 = 0; l2 < 2; l2++)
      hipLaunchKernelGGL(cedar_btab_build, dim3((n + 255) / 256), dim3(256), 0, s, d.btab, n, (uint32_t*)d.btab_mem, d.bmask, l2);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  (void)hipStreamDestroy(s);
  if (e != hipSuccess) {
    if (d.btab_mem) (void)hipFree(d.btab_mem);
    d.btab_mem = nullptr;
    return fail(e, "scope table build");
  }
  d.btab = (uint32_t*)d.btab_mem;
  d.bytes += bytes;
  return 0;
}

// (the whole blob: the host part rides along, ~15 % of a large image, so that a delta image can
// be applied on the device against it)
int dev_image_upload(int device, const Image& img, const uint8_t* blob, DevImage* out) {
  HIPCHK(hipSetDevice(device), "hipSetDevice");
  const size_t n = img.blob_len;
  void* base = nullptr;
  HIPCHK(hipMalloc(&base, std::max<size_t>(n, DS_ALIGN)), "hipMalloc image");
  if (hipMemcpy(base, blob, n, hipMemcpyHostToDevice) != hipSuccess) {
    (void)hipFree(base);
    g_err = "H2D image";
    return -5;
  }
  DevImage d;
  image_fields(img, device, base, 0, d);
  d.blob_len = n;
  if (const int rc = build_btab(img, d)) { (void)hipFree(base); return rc; }
  *out = d;
  return 0;
}

int dev_image_copy(int device, const Image& img, const DevImage& src, DevImage* out) {
  HIPCHK(hipSetDevice(device), "hipSetDevice");
  // the source's whole blob when it has it, else its region
  const bool whole = src.blob_len != 0 && src.origin == 0;
  const uint64_t origin = whole ? 0 : img.dev_begin;
  const size_t n = whole ? src.blob_len : img.dev_end - img.dev_begin;
  void* base = nullptr;
  HIPCHK(hipMalloc(&base, std::max<size_t>(n, DS_ALIGN)), "hipMalloc image");
  const uint8_t* from = (const uint8_t*)src.base + (origin - src.origin);
  const hipError_t e = device == src.device ? hipMemcpy(base, from, n, hipMemcpyDeviceToDevice)
                                            : hipMemcpyPeer(base, device, from, src.device, n);
  if (e != hipSuccess) {
    (void)hipFree(base);
    return fail(e, "peer copy of the image");
  }
  DevImage d;
  image_fields(img, device, base, origin, d);
  d.blob_len = whole ? n : 0;
  if (const int rc = build_btab(img, d)) { (void)hipFree(base); return rc; }
  *out = d;
  return 0;
}

int dev_image_adopt(int device, const Image& img, void* dev_blob, DevImage* out) {
  HIPCHK(hipSetDevice(device), "hipSetDevice");
  DevImage d;
  image_fields(img, device, dev_blob, 0, d);
  d.blob_len = img.blob_len;
  if (const int rc = build_btab(img, d)) return rc;  // the caller still owns dev_blob on failure
  *out = d;
  return 0;
}

// Delta images: one workgroup per piece (<= DL_PIECE bytes) copies it from the base blob or the
// literal bytes into the new blob, 16 bytes a lane when the piece's ends and both addresses allow
// (every piece of an unshifted section does), else 4, else 1. Pure copy: HBM-bound, ~2x the new
// blob's bytes at most; a one-CRD C5 delta moves ~110 MB through HBM in well under a millisecond.
__global__ void __launch_bounds__(256) cedar_blob_patch(const uint64_t* __restrict__ pc, const uint8_t* __restrict__ base,
                                                        const uint8_t* __restrict__ lit, uint8_t* __restrict__ out) {
  const uint64_t dst = pc[3 * (size_t)blockIdx.x], len = pc[3 * (size_t)blockIdx.x + 1], src = pc[3 * (size_t)blockIdx.x + 2];
  const uint8_t* s = (src & DL_LIT) ? lit + (src & ~DL_LIT) : base + src;
  uint8_t* d = out + dst;
  const uint64_t al = (uint64_t)(uintptr_t)s | (uint64_t)(uintptr_t)d | len;
  if ((al & 15) == 0) {
    const uint4* s4 = reinterpret_cast<const uint4*>(s);
    uint4* d4 = reinterpret_cast<uint4*>(d);
    for (uint64_t i = threadIdx.x; i < len / 16; i += 256) d4[i] = s4[i];
  } else if ((al & 3) == 0) {
    const uint32_t* s1 = reinterpret_cast<const uint32_t*>(s);
    uint32_t* d1 = reinterpret_cast<uint32_t*>(d);
    for (uint64_t i = threadIdx.x; i < len / 4; i += 256) d1[i] = s1[i];
  } else {
    for (uint64_t i = threadIdx.x; i < len; i += 256) d[i] = s[i];
  }
}

// the word fixups, after the pieces (a later launch on the same stream)
__global__ void __launch_bounds__(256) cedar_blob_fix(const uint32_t* __restrict__ fx, uint32_t n, uint32_t* __restrict__ out) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) out[fx[2 * i]] = fx[2 * i + 1];
}

int dev_blob_patch(int device, const DevImage& base, const uint64_t* pieces, size_t n_pieces, const uint8_t* lit,
                   size_t lit_len, const uint32_t* fix, size_t n_fix, size_t new_len, void** out) {
  HIPCHK(hipSetDevice(device), "hipSetDevice");
  if (!base.blob_len || base.origin != 0) { g_err = "the base image has no device blob"; return -2; }
  if (n_pieces > 0x7FFFFFFFu || n_fix > 0x7FFFFFFFu) { g_err = "delta too large"; return -2; }
  void* nb = nullptr;
  void* stage = nullptr;
  const size_t pbytes = n_pieces * 24, fbytes = n_fix * 8, sbytes = pbytes + fbytes + lit_len;
  HIPCHK(hipMalloc(&nb, std::max<size_t>(new_len, DS_ALIGN)), "hipMalloc image");
  hipError_t e = hipMalloc(&stage, std::max<size_t>(sbytes, 16));
  hipStream_t s = nullptr;
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipMemcpyAsync(stage, pieces, pbytes, hipMemcpyHostToDevice, s);
  if (e == hipSuccess && fbytes) e = hipMemcpyAsync((uint8_t*)stage + pbytes, fix, fbytes, hipMemcpyHostToDevice, s);
  if (e == hipSuccess && lit_len) e = hipMemcpyAsync((uint8_t*)stage + pbytes + fbytes, lit, lit_len, hipMemcpyHostToDevice, s);
  if (e == hipSuccess && n_pieces) {
    hipLaunchKernelGGL(cedar_blob_patch, dim3((uint32_t)n_pieces), dim3(256), 0, s, (const uint64_t*)stage,
                       (const uint8_t*)base.base, (const uint8_t*)stage + pbytes + fbytes, (uint8_t*)nb);
    e = hipGetLastError();
  }
  if (e == hipSuccess && n_fix) {
    hipLaunchKernelGGL(cedar_blob_fix, dim3((uint32_t)((n_fix + 255) / 256)), dim3(256), 0, s,
                       (const uint32_t*)((const uint8_t*)stage + pbytes), (uint32_t)n_fix, (uint32_t*)nb);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (s) (void)hipStreamDestroy(s);
  if (stage) (void)hipFree(stage);
  if (e != hipSuccess) {
    (void)hipFree(nb);
    return fail(e, "delta image patch");
  }
  *out = nb;
  return 0;
}

void dev_free(int device, void* p) {
  if (!p) return;
  (void)hipSetDevice(device);
  (void)hipFree(p);
}

// delta.h blob_word_mix, on the device (the same formula: the two must agree bit for bit)
__device__ __forceinline__ uint64_t dev_word_mix(uint64_t w, uint64_t i) {
  uint64_t z = w ^ (i * 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// blob_sum (delta.h) on the device: 16-byte loads (two words) over a grid-stride loop, a wave
// reduction, one 64-bit atomic add per wave; the zero-padded last word by thread 0
__global__ void __launch_bounds__(256) cedar_blob_sum(const uint8_t* __restrict__ p, uint64_t n, unsigned long long* __restrict__ out) {
  const uint64_t nq = n / 16;
  uint64_t acc = 0;
  for (uint64_t q = (uint64_t)blockIdx.x * 256 + threadIdx.x; q < nq; q += (uint64_t)gridDim.x * 256) {
    const uint4 v = reinterpret_cast<const uint4*>(p)[q];
    acc += dev_word_mix(((uint64_t)v.y << 32) | v.x, 2 * q) + dev_word_mix(((uint64_t)v.w << 32) | v.z, 2 * q + 1);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0)
    for (uint64_t o = nq * 16; o < n; o += 8) {
      uint64_t w = 0;
      for (uint64_t b = 0; b < 8 && o + b < n; b++) w |= (uint64_t)p[o + b] << (8 * b);
      acc += dev_word_mix(w, o / 8);
    }
  for (uint32_t o = 32; o > 0; o >>= 1) acc += (uint64_t)__shfl_xor((long long)acc, (int)o);
  if ((threadIdx.x & 63) == 0) atomicAdd(out, (unsigned long long)acc);
}

int dev_blob_sum(int device, const void* p, size_t n, uint64_t* out) {
  HIPCHK(hipSetDevice(device), "hipSetDevice");
  unsigned long long* d = nullptr;
  HIPCHK(hipMalloc((void**)&d, 8), "hipMalloc");
  hipError_t e = hipMemset(d, 0, 8);
  if (e == hipSuccess) {
    const uint64_t nq = n / 16;
    const uint32_t blocks = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(2048, (nq + 255) / 256));
    hipLaunchKernelGGL(cedar_blob_sum, dim3(blocks), dim3(256), 0, 0, (const uint8_t*)p, (uint64_t)n, d);
    e = hipGetLastError();
  }
  unsigned long long v = 0;
  if (e == hipSuccess) e = hipMemcpy(&v, d, 8, hipMemcpyDeviceToHost);
  (void)hipFree(d);
  if (e != hipSuccess) return fail(e, "blob checksum");
  *out = (uint64_t)v + (uint64_t)n;
  return 0;
}

int dev_to_host(int device, const void* src, size_t n, void* dst) {
  HIPCHK(hipSetDevice(device), "hipSetDevice");
  HIPCHK(hipMemcpy(dst, src, n, hipMemcpyDeviceToHost), "D2H");
  return 0;
}

void dev_image_free(DevImage* d) {
  if (d->device < 0) return;
  (void)hipSetDevice(d->device);
  if (d->base) (void)hipFree(d->base);
  if (d->btab_mem) (void)hipFree(d->btab_mem);
  *d = DevImage();
}

// A batch retired while its work may still run (dev_batch_retire): its blocks wait here until a
// host callback behind that work on its stream marks it drained; pool users then reap it.
struct Retired {
  DevBatch d;
  std::vector<DevSubset> held;
  std::atomic<bool> drained{false};
};
struct DevPool {
  int device = -1;
  std::mutex mu;
  std::multimap<size_t, void*> dev_free, host_free;  // size class -> idle block
  std::vector<std::pair<void*, bool>> owned;         // (block, pinned host)
  std::vector<Retired*> retired;                     // under mu
};
static void pool_reap(DevPool* p);

static size_t size_class(size_t n) {
  size_t c = (size_t)1 << 16;
  while (c < n) c <<= 1;
  return c;
}

static bool pinned_noncoherent() {
  static const bool on = [] { const char* e = std::getenv("CEDARGPU_PINNED_NONCOHERENT"); return e && *e == '1'; }();
  return on;
}

static int pool_get(DevPool* p, bool host, size_t n, void** out, size_t* cls) {
  *cls = size_class(n);
  pool_reap(p);
  {
    std::lock_guard<std::mutex> g(p->mu);
    auto& fl = host ? p->host_free : p->dev_free;
    auto it = fl.find(*cls);
    if (it != fl.end()) {
      *out = it->second;
      fl.erase(it);
      return 0;
    }
  }
  // CEDARGPU_PINNED_NONCOHERENT=1: pinned blocks the GPU may cache (A/B: the host's own reads of
  // the results). Kernels write zero-copy results into these blocks (DevBatch::zc), so that option
  // turns zero-copy off (dev_batch_upload): non-coherent blocks are then only DMA sources and targets.
  const unsigned pflags = pinned_noncoherent() ? hipHostMallocNonCoherent : hipHostMallocDefault;
  if (host) HIPCHK(hipHostMalloc(out, *cls, pflags), "hipHostMalloc");
  else HIPCHK(hipMalloc(out, *cls), "hipMalloc");
  std::lock_guard<std::mutex> g(p->mu);
  p->owned.emplace_back(*out, host);
  return 0;
}

static void pool_put(DevPool* p, bool host, void* blk, size_t cls) {
  if (!p || !blk) return;
  std::lock_guard<std::mutex> g(p->mu);
  (host ? p->host_free : p->dev_free).emplace(cls, blk);
}

// ---- pinned blocks for batch arrays (engine.h pinned_take) ----
// Process-wide, power-of-two classes PIN_MIN..PIN_MAX, recycled and never freed; on once a device
// context exists (the first dev_pool_create), so processes that only encode never touch the
// runtime. CEDARGPU_PINNED_ARRAYS=0 turns them off; CEDARGPU_PINNED_ARRAYS_MB caps the total
// (default 256 MB; past it arrays come from the heap and are staged as before).
namespace {
struct PinnedArrays {
  std::mutex mu;
  std::multimap<size_t, void*> idle;        // class -> block
  std::unordered_map<const void*, size_t> cls;  // block -> class
  size_t held = 0, cap = 0;
};
PinnedArrays& pinned_arrays() {
  static PinnedArrays* p = new PinnedArrays();  // (leaked: arrays may outlive static destruction)
  return *p;
}
std::atomic<bool> g_pin_on{false};
}  // namespace

void* pinned_take(size_t bytes) {
  if (!g_pin_on.load(std::memory_order_relaxed)) return nullptr;
  const size_t c = size_class(bytes);
  auto& pa = pinned_arrays();
  {
    std::lock_guard<std::mutex> g(pa.mu);
    auto it = pa.idle.find(c);
    if (it != pa.idle.end()) {
      void* b = it->second;
      pa.idle.erase(it);
      return b;
    }
    if (pa.held + c > pa.cap) return nullptr;
    pa.held += c;
  }
  void* b = nullptr;
  if (hipHostMalloc(&b, c, hipHostMallocDefault) != hipSuccess || !b) {
    (void)hipGetLastError();
    std::lock_guard<std::mutex> g(pa.mu);
    pa.held -= c;
    return nullptr;
  }
  std::lock_guard<std::mutex> g(pa.mu);
  pa.cls.emplace(b, c);
  return b;
}

bool pinned_give(void* p, size_t) {
  if (!p) return false;
  auto& pa = pinned_arrays();
  std::lock_guard<std::mutex> g(pa.mu);
  auto it = pa.cls.find(p);
  if (it == pa.cls.end()) return false;
  pa.idle.emplace(it->second, p);
  return true;
}

void pinned_stats(uint64_t* held_bytes, uint64_t* idle_blocks) {
  auto& pa = pinned_arrays();
  std::lock_guard<std::mutex> g(pa.mu);
  if (held_bytes) *held_bytes = pa.held;
  if (idle_blocks) *idle_blocks = pa.idle.size();
}

bool pinned_block(const void* p, size_t bytes) {
  if (!p) return false;
  auto& pa = pinned_arrays();
  std::lock_guard<std::mutex> g(pa.mu);
  auto it = pa.cls.find(p);
  return it != pa.cls.end() && bytes <= it->second;
}

int dev_pool_create(int device, DevPool** out) {
  *out = new (std::nothrow) DevPool();
  if (!*out) { g_err = "out of host memory"; return -1; }
  (*out)->device = device;
  static const bool pin = [] {
    const char* e = std::getenv("CEDARGPU_PINNED_ARRAYS");
    if (e && *e == '0') return false;
    const char* m = std::getenv("CEDARGPU_PINNED_ARRAYS_MB");
    pinned_arrays().cap = (size_t)(m ? std::max(0, std::atoi(m)) : 256) << 20;
    return true;
  }();
  if (pin) g_pin_on.store(true, std::memory_order_relaxed);
  return 0;
}

void dev_pool_destroy(DevPool* p) {
  if (!p) return;
  (void)hipSetDevice(p->device);
  (void)hipDeviceSynchronize();
  pool_reap(p);
  for (Retired* r : p->retired) delete r;  // (only on a device that never drained them)
  for (auto& o : p->owned) {
    if (o.second) (void)hipHostFree(o.first);
    else (void)hipFree(o.first);
  }
  delete p;
}

static bool split_on();

uint32_t dev_small_n() {  // (read per batch: tests cover both paths at small sizes)
  const char* e = std::getenv("CEDARGPU_SMALL_N");
  return e ? (uint32_t)std::atoi(e) : 2048u;
}

// One pinned staging block and one device block for the inputs (256-B aligned sections), one for
// the results; a batch costs two copies and a memset, and no allocation once the pool is warm.
// A few persistent helper threads for the staging copy of mid-sized batches (256 KB .. 8 MB: a
// 2,048-request batch stages 1.8 MB, ~95 us on one core): a copy is cut in STAGE_PARTS pieces, the
// helpers take all but the caller's own, the caller waits for them (a spawn per batch would cost
// what the copy saves). One copy at a time; a second caller copies alone.
namespace {
struct StagePool {
  static constexpr unsigned HELPERS = 3;
  std::mutex mu, busy;
  std::condition_variable cv;
  std::function<void(unsigned)> job;  // job(k) for part k = 1..HELPERS
  uint64_t gen = 0;
  std::atomic<unsigned> left{0};
  std::vector<std::thread> ts;
  StagePool() {
    for (unsigned t = 0; t < HELPERS; t++)
      ts.emplace_back([this, t] {
        uint64_t seen = 0;
        for (;;) {
          std::function<void(unsigned)> j;
          {
            std::unique_lock<std::mutex> g(mu);
            cv.wait(g, [&] { return gen != seen; });
            seen = gen;
            j = job;
          }
          j(t + 1);
          left.fetch_sub(1, std::memory_order_release);
        }
      });
    for (auto& t : ts) t.detach();  // process-lifetime helpers (never joined at exit)
  }
  // fn(k) for k = 0..HELPERS; false when another copy holds the pool (the caller runs them all)
  bool run(const std::function<void(unsigned)>& fn) {
    std::unique_lock<std::mutex> own(busy, std::try_to_lock);
    if (!own.owns_lock()) return false;
    left.store(HELPERS, std::memory_order_relaxed);
    {
      std::lock_guard<std::mutex> g(mu);
      job = fn;
      gen++;
    }
    cv.notify_all();
    fn(0);
    while (left.load(std::memory_order_acquire)) std::this_thread::yield();
    return true;
  }
};
StagePool& stage_pool() {
  static StagePool* p = new StagePool();  // (leaked: detached helpers outlive static destruction)
  return *p;
}
}  // namespace

static size_t scan_words(uint32_t n);

int dev_batch_upload(int device, const Batch& b, DevBatch* out, void* stream, DevPool* pool) {
  HIPCHK(hipSetDevice(device), "hipSetDevice");
  hipStream_t s = (hipStream_t)stream;
  DevBatch d;
  d.device = device;
  d.pool = pool;
  d.n = b.n();
  d.heap_words = b.heap.size();
  d.row_words = b.row_words;
  d.capr = b.capr;
  d.cape = b.cape;
  d.small = b.img->indexed && split_on() && b.n() && b.n() <= dev_small_n();
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  // the grouping keys travel only when the step groups the batch on the device
  const bool grp = b.dev_group && b.n() >= 2 && b.gkeys.size() == b.n();
  constexpr int NSEC = 6;
  const void* src[NSEC] = {b.heap.data(), b.req_base.data(), b.rows.data(), b.dev_str_off().data(), b.dev_str_bytes().data(), b.gkeys.data()};
  // (req_base stays on the host: the kernels read a request's block offset from its row, RW_BLK)
  const size_t len[NSEC] = {b.heap.size() * 4, 0, b.rows.size() * 4, b.dev_str_off().size() * 4, b.dev_str_bytes().size(),
                            grp ? b.gkeys.size() * 4 : 0};
  // Sections the encoder wrote into pinned blocks (engine.h pinned_take: a small batch's heap and
  // rows) are copied from there directly ("direct"); the rest is staged into one pinned block and
  // copied in one piece. Device layout: staged sections | (zero-copy) counters | direct sections.
  static const bool zc_on = !(std::getenv("CEDARGPU_ZERO_COPY") && *std::getenv("CEDARGPU_ZERO_COPY") == '0');
  d.zc = d.small && zc_on && !pinned_noncoherent();
  // (each copy costs ~10 us of queue gap on the device: the heap goes direct from PIN_MIN, the
  // other sections from 1 MB, CEDARGPU_DIRECT_MIN_KB; a 2,048-request C3 batch: its 1.8 MB heap
  // direct, 0.6 MB staged; submit -> results 173 -> 157 us, all four direct 159 us)
  static const size_t direct_min = [] { const char* e = std::getenv("CEDARGPU_DIRECT_MIN_KB"); return (size_t)(e ? std::max(64, std::atoi(e)) : 1024) << 10; }();
  bool direct[NSEC];
  for (int k = 0; k < NSEC; k++) direct[k] = len[k] >= (k == 0 ? PIN_MIN : direct_min) && pinned_block(src[k], len[k]);
  size_t off[NSEC], in_bytes = 0;
  for (int k = 0; k < NSEC; k++)
    if (!direct[k]) { off[k] = in_bytes; in_bytes += al(std::max<size_t>(len[k], 4)); }
  const size_t o_incnt = in_bytes;  // (zero-copy: the counters ride with the staged inputs)
  if (d.zc) in_bytes += al((FU_KINDS + 1) * 4);
  const size_t stage_in = in_bytes;
  for (int k = 0; k < NSEC; k++)
    if (direct[k]) { off[k] = in_bytes; in_bytes += al(len[k]); }
  const size_t n = std::max<uint32_t>(b.n(), 1);
  // The probe kernel writes only the deciding reason list (into reasons_f; reasons_p aliases it),
  // the policy-stream kernel both lists: an indexed image's first pass needs one array.
  const bool one_list = b.img->indexed != 0;
  // the worklist counters sit right behind res: the upload's one memset zeroes both
  const size_t o_res = 0, o_cnt = al(n * 2 * 4), o_rf = o_cnt + al((FU_KINDS + 1) * 4),
               o_rp = one_list ? o_rf : o_rf + al(n * d.capr * 4), o_er = o_rp + al(n * d.capr * 4);
  // On-device follow-up worklists. Entries: n / 32 (4..64) by default, or what the previous batch
  // on this image needed (the caller's hint), within a byte budget per worklist. Reasons per entry:
  // FU_BIG 256 unless the hint says otherwise (64..1024, the large stage's hit capacity), FU_OVF 64
  // (the probe kernel's), FU_GEN 64 unless hinted (..4096).
  const bool fu_on = !(std::getenv("CEDARGPU_FOLLOWUP") && *std::getenv("CEDARGPU_FOLLOWUP") == '0');
  const uint32_t fu_default = std::min<uint32_t>(64u, std::max<uint32_t>(4u, b.n() / 32u));
  const uint32_t capr_k[FU_KINDS] = {b.fu_capr_hint ? std::min<uint32_t>(1024u, std::max<uint32_t>(64u, b.fu_capr_hint)) : 256u,
                                     64u, std::min<uint32_t>(4096u, std::max<uint32_t>(64u, b.fu_capr_gen_hint))};
  // (FU_BIG: up to 256 MB, room for C3's 1M-request batches: ~43k many-hit requests of up to ~700
  // reasons each)
  const size_t budget_k[FU_KINDS] = {std::min<size_t>(256u << 20, std::max<size_t>(16u << 20, (size_t)b.n() * 2048)),
                                     std::min<size_t>(64u << 20, std::max<size_t>(8u << 20, (size_t)b.n() * 1024)),
                                     std::min<size_t>(64u << 20, std::max<size_t>(8u << 20, (size_t)b.n() * 1024))};
  // a grouped batch's pos_of (the gather kernel writes it; the host's accessors read through it)
  const bool with_pos = grp && !d.small;
  const size_t o_pos = o_er + al(n * d.cape * ERR_WORDS * 4);
  size_t o_fu = o_pos + (with_pos ? al(n * 4) : 0);
  size_t o_k[FU_KINDS][5];
  for (uint32_t k = 0; k < FU_KINDS; k++) {
    auto& f = d.fu[k];
    const bool probe_kind = k != FU_GEN;
    f.capr = capr_k[k];
    f.cape = 16;
    const size_t lists = probe_kind ? 1 : 2;
    const size_t entry = 4 * (1 + 2 + lists * (size_t)f.capr + (size_t)f.cape * ERR_WORDS);
    const uint32_t want = std::min<uint32_t>(b.n(), std::max(fu_default, b.fu_want[k]));
    f.cap = (fu_on && b.n() && !d.small && (!probe_kind || b.img->indexed)) ? (uint32_t)std::min<size_t>(want, budget_k[k] / entry) : 0u;
    if (d.small && k == FU_BIG && fu_on && b.img->n_pol() <= RANK_POL) {
      // the small path's overflow slots (KArgs::ovf_*, its SLIM merge): whole results of up to
      // 1,024 reasons and 32 errors for n / 8 requests (at least 8); only the slots a batch takes
      // travel back (dev_download_finish)
      f.capr = 1024;
      f.cape = 32;
      f.cap = std::min<uint32_t>(b.n(), std::max<uint32_t>(8u, b.n() / 8u));
    }
    o_k[k][0] = o_fu;                                        // ids
    o_k[k][1] = o_k[k][0] + al((size_t)f.cap * 4);           // res
    o_k[k][2] = o_k[k][1] + al((size_t)f.cap * 2 * 4);       // reasons_f
    o_k[k][3] = probe_kind ? o_k[k][2] : o_k[k][2] + al((size_t)f.cap * f.capr * 4);  // reasons_p
    o_k[k][4] = o_k[k][3] + al((size_t)f.cap * f.capr * 4);  // errors
    o_fu = o_k[k][4] + al((size_t)f.cap * f.cape * ERR_WORDS * 4);
  }
  d.out_bytes = o_fu;
  d.dl_bytes = (d.small && d.fu[FU_BIG].cap) ? o_k[FU_BIG][0] : o_fu;
  // Small batches: results written by the kernel into the pinned block (DevBatch::zc), behind the
  // staged inputs.
  const size_t o_zc = al(stage_in);
  int rc;
  if (b.img->lane_need > LANE_WORDS) {  // per-request lane scratch of the GLANE stream kernel
    const size_t lane_bytes = (size_t)n * b.img->lane_need * 4;
    if (lane_bytes > (8ull << 30)) {
      g_err = "batch needs " + std::to_string(lane_bytes >> 20) + " MB of lane scratch for this image's policies; submit smaller batches";
      return -7;  // CG_E_RANGE
    }
    if ((rc = pool_get(pool, false, lane_bytes, &d.lane_blk, &d.lane_cls))) return rc;
    d.lane = (uint32_t*)d.lane_blk;
  }
  if (b.img->indexed && split_on() && b.n() && !d.small) {  // the index scan's bucket lists
    if ((rc = pool_get(pool, false, scan_words(b.n()) * 4, &d.scan_blk, &d.scan_cls))) {
      pool_put(pool, false, d.lane_blk, d.lane_cls);
      return rc;
    }
    d.scan = (uint32_t*)d.scan_blk;
  }
  if (grp) {  // the device grouping's order, grouped rows, bucket counters and scan storage
    const size_t tb = group_temp_bytes(b.n());
    const size_t q = ((size_t)b.n() * 4 + 255) & ~(size_t)255, rq = group_gather() ? al((size_t)b.n() * b.row_words * 4) : 0;
    if (!tb) { g_err = "rocPRIM radix sort: no temporary storage size"; pool_put(pool, false, d.lane_blk, d.lane_cls); pool_put(pool, false, d.scan_blk, d.scan_cls); return -4; }
    if ((rc = pool_get(pool, false, 3 * q + rq + tb, &d.grp_blk, &d.grp_cls))) {
      pool_put(pool, false, d.lane_blk, d.lane_cls);
      pool_put(pool, false, d.scan_blk, d.scan_cls);
      return rc;
    }
    uint8_t* g8 = (uint8_t*)d.grp_blk;
    d.ord = (uint32_t*)g8;
    d.gkeys2 = (uint32_t*)(g8 + q);
    d.gvals = (uint32_t*)(g8 + 2 * q);
    d.grows = group_gather() ? (uint32_t*)(g8 + 3 * q) : nullptr;
    d.grp_temp = g8 + 3 * q + rq;
    d.grp_temp_bytes = tb;
  }
  if ((rc = pool_get(pool, false, in_bytes, &d.in_blk, &d.in_cls))) {
    pool_put(pool, false, d.lane_blk, d.lane_cls);
    pool_put(pool, false, d.scan_blk, d.scan_cls);
    pool_put(pool, false, d.grp_blk, d.grp_cls);
    return rc;
  }
  if (!d.zc && (rc = pool_get(pool, false, d.out_bytes, &d.out_blk, &d.out_cls))) {
    pool_put(pool, false, d.in_blk, d.in_cls);
    pool_put(pool, false, d.lane_blk, d.lane_cls);
    pool_put(pool, false, d.scan_blk, d.scan_cls);
    pool_put(pool, false, d.grp_blk, d.grp_cls);
    return rc;
  }
  if ((rc = pool_get(pool, true, d.zc ? o_zc + d.out_bytes : std::max(stage_in, d.out_bytes), &d.stage, &d.stage_cls))) {
    pool_put(pool, false, d.in_blk, d.in_cls);
    pool_put(pool, false, d.out_blk, d.out_cls);
    pool_put(pool, false, d.lane_blk, d.lane_cls);
    pool_put(pool, false, d.scan_blk, d.scan_cls);
    pool_put(pool, false, d.grp_blk, d.grp_cls);
    return rc;
  }
  uint8_t* st = (uint8_t*)d.stage;
  // Large batches (admission objects run to ~600 B per request) are staged by several threads:
  // one core's memcpy into pinned memory runs at ~10 GB/s.
  size_t total_len = 0;
  for (int k = 0; k < NSEC; k++) total_len += direct[k] ? 0 : len[k];
  const unsigned nt = total_len >= (8u << 20) ? std::min(8u, std::max(1u, std::thread::hardware_concurrency())) : 1u;
  uint8_t* in = (uint8_t*)d.in_blk;
  // byte range [t, t+1) / parts of the concatenated sections
  auto part_copy = [&](unsigned t, unsigned parts) {
    const size_t lo = total_len * t / parts, hi = total_len * (t + 1) / parts;
    size_t pos = 0;
    for (int k = 0; k < NSEC; k++) {
      if (direct[k]) continue;
      const size_t a = std::max(lo, pos), e = std::min(hi, pos + len[k]);
      if (a < e) std::memcpy(st + off[k] + (a - pos), (const uint8_t*)src[k] + (a - pos), e - a);
      pos += len[k];
    }
  };
  static const bool pooled = !(std::getenv("CEDARGPU_STAGE_POOL") && *std::getenv("CEDARGPU_STAGE_POOL") == '0');
  // Throughput batches (>= 64 MB to stage) are staged and copied in pieces: each piece's H2D copy
  // is enqueued as soon as its bytes are staged, so the staging memcpy runs under the copy engine's
  // transfer instead of ahead of it (CEDARGPU_STAGE_PIPE=0: stage everything, then one copy)
  static const bool pipe_on = !(std::getenv("CEDARGPU_STAGE_PIPE") && *std::getenv("CEDARGPU_STAGE_PIPE") == '0');
  const bool pipe = pipe_on && !d.zc && nt > 1 && total_len >= (64u << 20);
  if (pipe) {
    // (staged below, with the copies)
  } else if (nt <= 1 && pooled && total_len >= (256u << 10) &&
      stage_pool().run([&](unsigned t) { part_copy(t, StagePool::HELPERS + 1); })) {
    // (staged by the pool)
  } else if (nt <= 1) {
    for (int k = 0; k < NSEC; k++) if (len[k] && !direct[k]) std::memcpy(st + off[k], src[k], len[k]);
  } else {
    auto part = [&](unsigned t) {  // byte range [t, t+1) / nt of the concatenated sections
      const size_t lo = total_len * t / nt, hi = total_len * (t + 1) / nt;
      size_t pos = 0;
      for (int k = 0; k < NSEC; k++) {
        if (direct[k]) continue;
        const size_t a = std::max(lo, pos), b = std::min(hi, pos + len[k]);
        if (a < b) std::memcpy(st + off[k] + (a - pos), (const uint8_t*)src[k] + (a - pos), b - a);
        pos += len[k];
      }
    };
    std::vector<std::thread> ts;
    for (unsigned t = 1; t < nt; t++) ts.emplace_back(part, t);
    part(0);
    for (auto& th : ts) th.join();
  }
  uint8_t* o = (uint8_t*)d.out_blk;
  if (d.zc) {
    void* dp = nullptr;
    if (hipHostGetDevicePointer(&dp, d.stage, 0) != hipSuccess || !dp) {
      g_err = "hipHostGetDevicePointer: pinned block not mapped for the device";
      pool_put(pool, false, d.in_blk, d.in_cls);
      pool_put(pool, true, d.stage, d.stage_cls);
      pool_put(pool, false, d.lane_blk, d.lane_cls);
      pool_put(pool, false, d.scan_blk, d.scan_cls);
      pool_put(pool, false, d.grp_blk, d.grp_cls);
      return -4;
    }
    o = (uint8_t*)dp + o_zc;
    d.zc_out = st + o_zc;
    d.zc_cnt = (uint32_t*)(st + o_zc + o_cnt);
    std::memset(st + o_incnt, 0, (FU_KINDS + 1) * 4);  // the counters (they travel with the inputs)
    std::memset(d.zc_out + o_res, 0, n * 2 * 4);        // res: RF_VALID clear until written
  }
  d.heap = (uint32_t*)(in + off[0]);
  d.rows = (uint32_t*)(in + off[2]);
  d.bstr_off = (uint32_t*)(in + off[3]);
  d.bstr_bytes = in + off[4];
  if (grp) d.gkeys = (const uint32_t*)(in + off[5]);
  d.res = (uint32_t*)(o + o_res);
  d.reasons_f = (uint32_t*)(o + o_rf);
  d.reasons_p = (uint32_t*)(o + o_rp);
  d.errs = (uint32_t*)(o + o_er);
  d.pos_of = with_pos ? (uint32_t*)(o + o_pos) : nullptr;
  d.fu_cnt = (uint32_t*)(d.zc ? in + o_incnt : o + o_cnt);
  for (uint32_t k = 0; k < FU_KINDS; k++) {
    auto& f = d.fu[k];
    f.ids = (uint32_t*)(o + o_k[k][0]);
    f.res = (uint32_t*)(o + o_k[k][1]);
    f.rf = (uint32_t*)(o + o_k[k][2]);
    f.rp = (uint32_t*)(o + o_k[k][3]);
    f.er = (uint32_t*)(o + o_k[k][4]);
  }
  d.bytes = in_bytes + d.out_bytes;
  d.stream = stream;
  d.pending = true;
  // (set before the copy into *out: ~cg_batch reads out->direct to keep the direct sources alive
  // past a close while in flight, DevBatch::keep)
  d.direct = false;
  for (int k = 0; k < NSEC; k++) d.direct = d.direct || direct[k];
  if (b.prof)
    for (auto& e : d.pev) {
      hipEvent_t ev;
      HIPCHK(hipEventCreate(&ev), "profile event");
      e = (void*)ev;
    }
  *out = d;  // blocks owned by the batch from here on (freed by dev_batch_free on any error)
  if (d.pev[0]) HIPCHK(hipEventRecord((hipEvent_t)d.pev[0], s), "event record");
  // (one copy below 64 MB: staging in pieces with an H2D per piece, to overlap the two, made
  // 1-2k-request batches 0.06-0.07 ms slower on the box, gpurun_out/r04flat3)
  if (pipe) {
    // pieces of <= 16 MB of the staged sections, in order; nt workers take (piece, part) items in
    // order and this thread enqueues each piece's copy once all its parts are staged
    constexpr size_t PIECE = 16u << 20;
    struct Piece { int k; size_t a, b; };
    std::vector<Piece> pcs;
    for (int k = 0; k < NSEC; k++)
      if (len[k] && !direct[k])
        for (size_t a = 0; a < len[k]; a += PIECE) pcs.push_back({k, a, std::min(len[k], a + PIECE)});
    std::unique_ptr<std::atomic<uint32_t>[]> done(new std::atomic<uint32_t>[pcs.size()]);
    for (size_t i = 0; i < pcs.size(); i++) done[i].store(0, std::memory_order_relaxed);
    std::atomic<size_t> next{0};
    const size_t items = pcs.size() * nt;
    auto work = [&] {
      for (size_t it; (it = next.fetch_add(1, std::memory_order_relaxed)) < items;) {
        const Piece& pc = pcs[it / nt];
        const size_t t = it % nt, n_ = pc.b - pc.a, lo = pc.a + n_ * t / nt, hi = pc.a + n_ * (t + 1) / nt;
        if (lo < hi) std::memcpy(st + off[pc.k] + lo, (const uint8_t*)src[pc.k] + lo, hi - lo);
        done[it / nt].fetch_add(1, std::memory_order_release);
      }
    };
    std::vector<std::thread> ts;
    for (unsigned t = 0; t < nt; t++) ts.emplace_back(work);
    hipError_t ce = hipSuccess;
    for (size_t i = 0; i < pcs.size(); i++) {
      while (done[i].load(std::memory_order_acquire) < nt) std::this_thread::yield();
      const Piece& pc = pcs[i];
      if (ce == hipSuccess) ce = hipMemcpyAsync(in + off[pc.k] + pc.a, st + off[pc.k] + pc.a, pc.b - pc.a, hipMemcpyHostToDevice, s);
    }
    for (auto& th : ts) th.join();
    HIPCHK(ce, "hipMemcpyAsync H2D (piece)");
  } else {
    HIPCHK(hipMemcpyAsync(in, st, stage_in, hipMemcpyHostToDevice, s), "hipMemcpyAsync H2D");
  }
  // (the direct sources belong to the host batch, which keeps them until this stream has drained:
  // cg_batch's destructor hands them to the retired batch, DevBatch::keep)
  for (int k = 0; k < NSEC; k++)
    if (direct[k]) HIPCHK(hipMemcpyAsync(in + off[k], src[k], len[k], hipMemcpyHostToDevice, s), "hipMemcpyAsync H2D (pinned array)");
  if (!d.zc) HIPCHK(hipMemsetAsync(d.res, 0, o_rf, s), "memset res");  // (and the worklist counters)
  if (d.pev[1]) HIPCHK(hipEventRecord((hipEvent_t)d.pev[1], s), "event record");
  return 0;
}

bool dev_batch_profile(const DevBatch& b, float* h2d_ms, float* step_ms, float* d2h_ms) {
  if (!b.pev[0] || !b.pev[3]) return false;
  (void)hipSetDevice(b.device);
  float t[3] = {0.f, 0.f, 0.f};
  for (int k = 0; k < 3; k++)
    if (hipEventElapsedTime(&t[k], (hipEvent_t)b.pev[k], (hipEvent_t)b.pev[k + 1]) != hipSuccess) return false;
  *h2d_ms = t[0];
  *step_ms = t[1];
  *d2h_ms = t[2];
  return true;
}

void dev_batch_free(DevBatch* d) {
  if (d->device < 0) return;
  (void)hipSetDevice(d->device);
  if (d->pending && d->stream) {
    // work on the batch's blocks may still run (submitted, never waited): drain its stream first
    hipEvent_t e;
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess) {
      (void)hipEventRecord(e, (hipStream_t)d->stream);
      (void)hipEventSynchronize(e);
      (void)hipEventDestroy(e);
    } else {
      (void)hipDeviceSynchronize();
    }
  }
  if (d->done) (void)hipEventDestroy((hipEvent_t)d->done);
  for (auto e : d->pev)
    if (e) (void)hipEventDestroy((hipEvent_t)e);
  if (d->pool) {
    pool_put(d->pool, false, d->in_blk, d->in_cls);
    pool_put(d->pool, false, d->out_blk, d->out_cls);
    pool_put(d->pool, true, d->stage, d->stage_cls);
    pool_put(d->pool, false, d->lane_blk, d->lane_cls);
    pool_put(d->pool, false, d->scan_blk, d->scan_cls);
    pool_put(d->pool, false, d->grp_blk, d->grp_cls);
  }
  if (d->req_idx) (void)hipFree(d->req_idx);
  *d = DevBatch();
}

// host callback behind a retired batch's work: no HIP calls here (HIP forbids them in callbacks)
static void retired_drained(void* r) { static_cast<Retired*>(r)->drained.store(true, std::memory_order_release); }

static void pool_reap(DevPool* p) {
  std::vector<Retired*> done;
  {
    std::lock_guard<std::mutex> g(p->mu);
    if (p->retired.empty()) return;
    auto keep = p->retired.begin();
    for (Retired* r : p->retired) {
      if (r->drained.load(std::memory_order_acquire)) done.push_back(r);
      else *keep++ = r;
    }
    p->retired.erase(keep, p->retired.end());
  }
  for (Retired* r : done) {
    r->d.pending = false;  // its stream passed the callback: nothing of it runs any more
    dev_batch_free(&r->d);
    for (auto& j : r->held) dev_subset_release(&j);
    delete r;
  }
}

void dev_batch_retire(DevBatch* d, std::vector<DevSubset>& held) {
  bool busy = d->pending && d->stream;
  for (auto& j : held)
    if (j.done && hipEventQuery((hipEvent_t)j.done) == hipErrorNotReady) busy = true;
  DevPool* pool = d->pool;
  if (!busy || !pool || d->device < 0) {
    dev_batch_free(d);
    for (auto& j : held) dev_subset_release(&j);
    held.clear();
    return;
  }
  (void)hipSetDevice(d->device);
  Retired* r = new (std::nothrow) Retired();
  if (r) {
    r->d = *d;
    r->held.swap(held);
    // host re-runs run on the context's re-run stream: the batch's stream waits for every one still
    // in flight, so the one callback behind it covers them all
    bool ordered = true;
    for (auto& j : r->held)
      if (j.done && hipEventQuery((hipEvent_t)j.done) == hipErrorNotReady)
        ordered = ordered && hipStreamWaitEvent((hipStream_t)d->stream, (hipEvent_t)j.done, 0) == hipSuccess;
    if (ordered && hipLaunchHostFunc((hipStream_t)d->stream, retired_drained, r) == hipSuccess) {
      {
        std::lock_guard<std::mutex> g(pool->mu);
        pool->retired.push_back(r);
      }
      *d = DevBatch();
      return;
    }
    held.swap(r->held);
    delete r;
  }
  dev_batch_free(d);  // no callback could be enqueued: fall back to draining the stream here
  for (auto& j : held) dev_subset_release(&j);
  held.clear();
}

static size_t lds_bytes(const DevImage& img) { return (size_t)std::max<uint32_t>(img.n_hot, 1) * BLOCK * sizeof(uint2); }

// Worklists of the on-device follow-up (device.h FuKind): every request the first pass left
// unfinished (RF_OVERFLOW), by what finishes it, in any order. cnt[k] counts them all; entries
// past cap[k] are left to the host re-run.
struct FuLists {
  uint32_t* ids[FU_KINDS];
  uint32_t cap[FU_KINDS];
};
// A block covers GATHER_ITEMS * 256 requests (coalesced strides of 256) in two passes over their
// result words: count per worklist, block-wide exclusive scan in LDS, ONE atomicAdd per worklist
// per block for its base, then write the ids. (One atomic per unfinished request serialised on
// three L2 addresses: 153 us for the 14.7k of a 1M-request C3 batch.)
constexpr uint32_t GATHER_ITEMS = 4;  // (1,024 blocks per 1M requests; 16, 256 blocks: 0.030 vs 0.021 ms, gpurun_out/r06t3)
__device__ __forceinline__ uint32_t fu_kind(uint32_t fl, uint32_t indexed) {
  if (!(fl & RF_OVERFLOW)) return FU_KINDS;
  return ((fl & RF_GENERAL) || !indexed) ? FU_GEN : (fl & RF_BIG) ? FU_BIG : FU_OVF;
}
// (grouped batches: every position i also inverts the order, pos_of[ord[i]] = i, for the host's
// result accessors, engine.h Batch::slot; the order's reads are coalesced, the scattered 4-byte
// writes are the one scatter left in the step)
__global__ void __launch_bounds__(256) cedar_fu_gather(const uint32_t* __restrict__ res, uint32_t n, uint32_t indexed,
                                                       uint32_t* __restrict__ cnt, FuLists wl,
                                                       const uint32_t* __restrict__ ord, uint32_t* __restrict__ pos_of) {
  __shared__ uint32_t scan[FU_KINDS][256];
  __shared__ uint32_t base[FU_KINDS];
  const uint32_t t = threadIdx.x;
  const size_t b0 = (size_t)blockIdx.x * GATHER_ITEMS * 256;
  uint32_t c[FU_KINDS] = {0, 0, 0};
  for (uint32_t k = 0; k < GATHER_ITEMS; k++) {
    const size_t i = b0 + (size_t)k * 256 + t;
    const uint32_t q = i < n ? fu_kind(res[2 * i] >> 16, indexed) : FU_KINDS;
    if (q < FU_KINDS) c[q]++;
    if (pos_of && i < n) pos_of[ord[i]] = (uint32_t)i;
  }
  for (uint32_t q = 0; q < FU_KINDS; q++) scan[q][t] = c[q];
  __syncthreads();
  for (uint32_t o = 1; o < 256; o <<= 1) {  // inclusive Hillis-Steele scan, three lists at once
    uint32_t v[FU_KINDS];
    for (uint32_t q = 0; q < FU_KINDS; q++) v[q] = t >= o ? scan[q][t - o] : 0u;
    __syncthreads();
    for (uint32_t q = 0; q < FU_KINDS; q++) scan[q][t] += v[q];
    __syncthreads();
  }
  if (t < FU_KINDS) base[t] = scan[t][255] ? atomicAdd(cnt + t, scan[t][255]) : 0u;
  __syncthreads();
  uint32_t pos[FU_KINDS];
  for (uint32_t q = 0; q < FU_KINDS; q++) pos[q] = base[q] + scan[q][t] - c[q];
  for (uint32_t k = 0; k < GATHER_ITEMS; k++) {
    const size_t i = b0 + (size_t)k * 256 + t;
    const uint32_t q = i < n ? fu_kind(res[2 * i] >> 16, indexed) : FU_KINDS;
    if (q < FU_KINDS) {
      if (pos[q] < wl.cap[q]) wl.ids[q][pos[q]] = (uint32_t)i;
      pos[q]++;
    }
  }
}

// the scan lists' layout in DevBatch::scan (KArgs::scan): n count words | a list total per wave of
// 8 positions | a WAVE_CAP-pair list per wave
static size_t scan_words(uint32_t n) {
  const size_t nw = ((size_t)n + 7) / 8;
  return (((size_t)n + 63) & ~(size_t)63) + ((nw + 63) & ~(size_t)63) + nw * 2 * WAVE_CAP;
}
static void set_scan(KArgs& k, const DevBatch& b) {
  const size_t nw = ((size_t)b.n + 7) / 8;
  k.scan = b.scan;
  k.scan_tot = b.scan + (((size_t)b.n + 63) & ~(size_t)63);
  k.scan_list = k.scan_tot + ((nw + 63) & ~(size_t)63);
  k.scan_n = b.n;
}

static KArgs make_args(const DevImage& img, const DevBatch& b, const uint32_t* req_idx, uint32_t n, uint32_t* res,
                       uint32_t* rf, uint32_t* rp, uint32_t* er, uint32_t capr, uint32_t cape) {
  KArgs k;
  k.pstream = img.pstream; k.tier_cend = img.tier_cend; k.chunks = img.chunks; k.cpool = img.cpool;
  k.gstr_off = img.gstr_off; k.gstr_bytes = img.gstr_bytes; k.hot = img.hot;
  k.heap = b.heap; k.req_idx = req_idx;
  k.bstr_off = b.bstr_off; k.bstr_bytes = b.bstr_bytes;
  k.res = res; k.reasons_f = rf; k.reasons_p = rp; k.errs = er;
  k.n_pol = img.n_pol; k.n_tiers = img.n_tiers; k.n_gstr = img.n_gstr; k.n_hot = img.n_hot;
  k.act = img.act; k.n_act = img.n_act; k.amask_ok = img.amask_ok;
  k.n_req = n; k.capr = capr; k.cape = cape;
  k.btab = img.btab; k.bfilt = img.bfilt; k.bstream = img.bstream; k.bmask = img.bmask; k.fmask = img.fmask;
  k.sctx = img.sctx; k.sbits = img.sbits; k.svals = img.svals; k.sctx_mask = img.sctx_mask; k.sbits_words = img.sbits_words;
  // the context filter (CEDARGPU_CTX_BLOOM=0: probe every context, A/B)
  static const bool ctx_bloom = !(std::getenv("CEDARGPU_CTX_BLOOM") && *std::getenv("CEDARGPU_CTX_BLOOM") == '0');
  k.sbloom = ctx_bloom ? img.sbloom : nullptr;
  k.n_kent = img.n_kent;
  k.bad_kidx = b.fu_cnt ? b.fu_cnt + FU_KINDS : nullptr;
  k.l2_vmask = img.l2_vmask; k.l2_lmask = img.l2_lmask;
  k.rows = b.rows; k.row_words = b.row_words; k.combo_mask = img.combo_mask;
  k.srows = img.srows; k.shash = reinterpret_cast<const uint4*>(img.shash); k.n_static = img.n_static; k.smask = img.smask;
  k.lane = b.lane; k.lane_stride = img.lane_need;
  k.hlists = img.cslot_mask;  // (DevImage::cslot_mask: the image's list slots)
  // like words staged behind the hot values while both fit the probe kernel's hot rows (32 entries;
  // CEDARGPU_LIKE_STAGE=0: never, A/B): else AK_LIKEI reads the string's bytes
  // (read on every call, as CEDARGPU_SMALL_N is: tests switch it within one process)
  const char* ls_env = std::getenv("CEDARGPU_LIKE_STAGE");
  const bool like_stage = !(ls_env && *ls_env == '0');
  static const uint32_t xcd_chunk = [] { const char* e = std::getenv("CEDARGPU_XCD_CHUNK"); return e ? (uint32_t)std::atoi(e) : 0u; }();
  k.xcd_chunk = xcd_chunk;
  static const uint32_t park = [] { const char* e = std::getenv("CEDARGPU_PARK_ATOMS"); return e && std::atoi(e) == 2 ? 2u : 4u; }();
  k.park = park;
  // CEDARGPU_CLASS_SLOTS=0: every member of a duplicate class takes a hit slot (A/B)
  static const bool cls_slots = !(std::getenv("CEDARGPU_CLASS_SLOTS") && *std::getenv("CEDARGPU_CLASS_SLOTS") == '0');
  k.cls = cls_slots && img.cls_compact ? 1u : 0u;
  k.lslot = img.lslot_mask;
  k.like_off = img.like_off;
  k.like_base = (like_stage && img.lslot_mask && img.n_hot + 3u * (uint32_t)__builtin_popcount(img.lslot_mask) <= NHOT) ? img.n_hot : 0xFFFFFFFFu;
  // off by default: the scope table is sized for ~1.06-slot chains, where a miss costs one slot load
  // and the filter only adds a round trip in front of every hit (profiles/r02/ab_slack)
  static const uint32_t l1filt = [] { const char* e = std::getenv("CEDARGPU_L1_FILTER"); return (e && *e == '1') ? 1u : 0u; }();
  k.l1filt = l1filt;
  // off by default: the level-1 entry's bloom already passes only likely keys (+2 %, profiles/r02/ab_mix)
  static const uint32_t l2filt = [] { const char* e = std::getenv("CEDARGPU_L2_FILTER"); return (e && *e == '1') ? 1u : 0u; }();
  k.l2filt = l2filt;
  static const uint32_t slot_split = [] { const char* e = std::getenv("CEDARGPU_SLOT_SPLIT"); return (e && *e == '1') ? 1u : 0u; }();
  k.slot_split = slot_split;
  static const uint32_t scan_lds = [] { const char* e = std::getenv("CEDARGPU_SCAN_LDS"); return (e && *e == '0') ? 0u : 1u; }();
  k.scan_lds = scan_lds;
  // on by default: the two-level bitset pass lists ~7.6 exact keys per C3 request instead of
  // enumerating ~62 level-1 keys and their level-2 follow-ups (scan 1.02 -> 0.85 ms per 1M,
  // profiles/r03/ab10); CEDARGPU_SCAN_FILT=0 enumerates (A/B)
  static const uint32_t scan_filt = [] { const char* e = std::getenv("CEDARGPU_SCAN_FILT"); return (e && *e == '0') ? 0u : 1u; }();
  k.scan_filt = scan_filt;
  // 48: C3 DAG 4.91e8 decisions/s at 32..96 alike; a list of 24 that sent every longer one to the
  // large stage measured 4.58e8 (43,485 large-stage requests instead of 25,005; profiles/r02/ab_scan_cap)
  static const uint32_t scan_big = [] { const char* e = std::getenv("CEDARGPU_SCAN_BIG"); return e ? (uint32_t)std::atoi(e) : 48u; }();
  static const uint32_t scan_heavy = [] { const char* e = std::getenv("CEDARGPU_SCAN_HEAVY"); return e ? (uint32_t)std::atoi(e) : 128u; }();
  k.scan_heavy = std::min<uint32_t>(scan_heavy, 1u << 20);  // (FP_PRE: a round's candidates below 2^24)
  static const uint32_t cnt_rank = [] { const char* e = std::getenv("CEDARGPU_CNT_RANK"); return e ? (uint32_t)std::atoi(e) : 32u; }();
  k.cnt_rank = cnt_rank;
  k.scan_big = scan_big;
  k.stats = nullptr;
  k.n_dev = nullptr;
  // a grouped batch's order (the device sort's, set by the step's grouping): every kernel of the
  // step and of its host re-runs finds the row of position p at ord[p]
  k.ord = b.small ? nullptr : b.ord;
  k.grows = (k.ord && group_gather()) ? b.grows : nullptr;
  k.scan = nullptr;
  k.scan_tot = k.scan_list = nullptr;
  k.scan_n = 0;
  k.ovf_cnt = nullptr;
  k.ovf_ids = k.ovf_res = k.ovf_rf = k.ovf_er = nullptr;
  k.ovf_cap = k.ovf_capr = k.ovf_cape = 0;
  return k;
}

// Launches the evaluation of n requests: the request-per-wave kernel over the scope index when the
// image is fully indexed, else the request-per-lane policy-stream kernel.
// Probe-kernel segment width (lanes per request): 8 by default, 8 requests per wave (on the C3
// group-DAG workload 2.94e8 decisions/s against 2.21e8 with 16 lanes: a request's ~60 level-1
// probes are dependent-latency chains, and more requests in flight per wave hide them;
// profiles/r02/ab_seg8); CEDARGPU_PROBE_SEG=16 / 32 / 64 for comparisons.
// Per-phase timing of a step (dev_time_split): while set, the step records an event at the end of
// each phase (device.h STEP_PHASES) on its stream.
static thread_local hipEvent_t* t_marks = nullptr;
static void mark(uint32_t phase, hipStream_t s) {
  if (t_marks) (void)hipEventRecord(t_marks[phase + 1], s);
}

static bool split_on() {
  static const bool on = !(std::getenv("CEDARGPU_SPLIT") && *std::getenv("CEDARGPU_SPLIT") == '0');
  return on;
}
static uint32_t probe_seg() {
  static const uint32_t seg = [] {
    const char* e = std::getenv("CEDARGPU_PROBE_SEG");
    const uint32_t v = e ? (uint32_t)std::atoi(e) : 8u;
    return (v == 16u || v == 32u || v == 64u) ? v : 8u;
  }();
  return seg;
}

// big: the re-run variant for requests with more hits than the default stage (one request per
// wave, 1024 hits staged)
// Minimum waves per SIMD the probe kernel is register-allocated for. 16 lanes: 4 (128 VGPRs, a few
// spilled dwords) measured +15 % over the unconstrained allocation (3 waves) and ahead of 5.
// 8 lanes: 3 (168 VGPRs, no spills; the 8-request LDS region allows no more) measured 2.94e8
// against 2.44e8 when forced to 4; CEDARGPU_PROBE_OCC selects the others for comparisons.
static uint32_t probe_occ() {
  static const uint32_t occ = [] {
    const char* e = std::getenv("CEDARGPU_PROBE_OCC");
    const uint32_t d = probe_seg() == 8 ? 3u : 4u;
    const uint32_t v = e ? (uint32_t)std::atoi(e) : d;
    return (v == 1u || v == 3u || v == 4u || v == 5u) ? v : d;
  }();
  return occ;
}

// CEDARGPU_PROBE_STATS=1: every default-variant launch runs the counting variant, synchronously,
// and prints its per-request work profile to stderr (profiling only).
static bool probe_stats() {
  static const bool on = std::getenv("CEDARGPU_PROBE_STATS") != nullptr;
  return on;
}

// Waves per block of the default probe kernel: 1 (one-wave blocks: a finished wave's slot is
// reused at once; 4-wave blocks hold their resources until the slowest wave ends — 770M vs 626M
// decisions/s, profiles/r01/ab_v9/wpb_*). CEDARGPU_PROBE_WPB = 2 / 4 for comparisons.
static uint32_t probe_wpb() {
  static const uint32_t w = [] {
    const char* e = std::getenv("CEDARGPU_PROBE_WPB");
    const uint32_t v = e ? (uint32_t)std::atoi(e) : 1u;
    return (v == 2u || v == 4u) ? v : 1u;
  }();
  return w;
}

// The first pass of an indexed image runs split (cedar_scan_kernel, then the probe kernel's SPLIT
// variant over the buckets it found); CEDARGPU_SPLIT=0 runs the fused probe kernel instead.
// the large stage's register target: 3 waves per SIMD (168 VGPRs), which its LDS (3 four-wave
// blocks per CU) also allows
constexpr uint32_t BIG_MINW = 3;
// ... and its SLIM form (images of <= RANK_POL policies): 8,960 B of LDS lets 4 waves per SIMD in,
// so it asks for them (128 VGPRs); CEDARGPU_BIG_SLIM=0 keeps the hm form, =3 the SLIM form at 3 (A/B)
constexpr uint32_t BIG_SLIM_MINW = 4;
static uint32_t big_slim(const KArgs& k) {  // 0: the hm form; else the SLIM form's waves per SIMD
  static const uint32_t on = [] { const char* e = std::getenv("CEDARGPU_BIG_SLIM"); return e ? (uint32_t)std::atoi(e) : BIG_SLIM_MINW; }();
  return k.n_pol <= RANK_POL ? on : 0u;
}
// the probe kernel's per-wave STATS counters (cedar_probe_kernel), summed
static void print_probe_stats(const char* what, const std::vector<unsigned long long>& h, size_t nw) {
  double sum[16] = {0};
  std::vector<unsigned long long> tot(nw);
  for (size_t w = 0; w < nw; w++) {
    for (int i = 0; i < 16; i++) sum[i] += (double)h[w * 16 + i];
    tot[w] = h[w * 16 + 12] + h[w * 16 + 13] + h[w * 16 + 14] + h[w * 16 + 15];
  }
  // the launch's makespan if its waves took these cycles, handed in launch order (and, for
  // comparison, longest first) to 256 CUs x 16 wave slots as each slot frees: how much of the
  // kernel's time a dispatch order could win back from its slowest waves
  auto makespan = [&](const std::vector<unsigned long long>& d) {
    std::priority_queue<unsigned long long, std::vector<unsigned long long>, std::greater<unsigned long long>> free_at;
    for (int i = 0; i < 256 * 16; i++) free_at.push(0);
    unsigned long long end = 0;
    for (unsigned long long x : d) {
      const unsigned long long t = free_at.top() + x;
      free_at.pop();
      free_at.push(t);
      end = std::max(end, t);
    }
    return end;
  };
  double all = 0;
  size_t idle = 0;  // waves whose requests have no candidate head at all
  for (size_t w = 0; w < nw; w++) idle += h[w * 16 + 6] == 0;
  for (unsigned long long x : tot) all += (double)x;
  const unsigned long long in_order = makespan(tot);
  const unsigned long long reversed = makespan(std::vector<unsigned long long>(tot.rbegin(), tot.rend()));
  std::sort(tot.begin(), tot.end());
  const unsigned long long longest_first = makespan(std::vector<unsigned long long>(tot.rbegin(), tot.rend()));
  std::fprintf(stderr, "%s dispatch: makespan in launch order %llu, reversed %llu, longest first %llu, bound %.0f (cycles); "
               "waves without candidates %.3f\n", what, in_order, reversed, longest_first, all / (256.0 * 16.0),
               nw ? (double)idle / (double)nw : 0.0);
  const double r = sum[0] > 0 ? sum[0] : 1.0, W = (double)nw;
  std::fprintf(stderr,
               "%s stats: requests %.0f | per request: L1 keys %.2f found %.2f | L2 probes %.2f found %.2f | "
               "slots %.2f | heads %.2f scope-ok %.2f | atoms %.2f | hits %.2f | stage flushes %.2f | "
               "candidate passes %.2f\n  per wave cycles: load %.0f probe %.0f candidates %.0f merge %.0f | total p50 %llu "
               "p90 %llu p99 %llu max %llu\n",
               what, sum[0], sum[1] / r, sum[2] / r, sum[3] / r, sum[4] / r, sum[5] / r, sum[6] / r, sum[7] / r, sum[8] / r,
               sum[9] / r, sum[10] / r, sum[11] / r, sum[12] / W, sum[13] / W, sum[14] / W, sum[15] / W, tot[nw / 2],
               tot[nw * 9 / 10], tot[nw * 99 / 100], tot[nw - 1]);
}

static void launch_probe(const KArgs& k, uint32_t n, hipStream_t s, bool big = false) {
  // (a follow-up over scanned requests runs on the large stage: the pooled candidate pass reads
  // whole wave lists of the first pass, by its own launch position)
  if (k.scan && k.req_idx) big = true;
  if (big && k.scan) {  // the large stage over the scan's buckets (probing only past SCAN_CAP)
    // one-wave blocks: a finished request's wave slot and LDS return at once (C3 DAG 4.996e8 vs
    // 4.919e8 with 4-wave blocks, profiles/r02/ab_big_occ)
    static const uint32_t bw = [] { const char* e = std::getenv("CEDARGPU_BIG_WPB"); return e ? (uint32_t)std::atoi(e) : 1u; }();
    static const bool bstats = std::getenv("CEDARGPU_BIG_STATS") != nullptr;
    if (bstats) {  // the large stage's work counters (profiling)
      unsigned long long* d = nullptr;
      if (hipMalloc((void**)&d, (size_t)n * 16 * 8) == hipSuccess) {
        KArgs ks = k;
        ks.stats = d;
        (void)hipMemsetAsync(d, 0, (size_t)n * 16 * 8, s);
        if (big_slim(k) == BIG_SLIM_MINW) hipLaunchKernelGGL((cedar_probe_kernel<64, 1024, BIG_SLIM_MINW, true, 1, true, true>), dim3(n), dim3(64), 0, s, ks);
        else if (big_slim(k)) hipLaunchKernelGGL((cedar_probe_kernel<64, 1024, BIG_MINW, true, 1, true, true>), dim3(n), dim3(64), 0, s, ks);
        else hipLaunchKernelGGL((cedar_probe_kernel<64, 1024, BIG_MINW, true, 1, true>), dim3(n), dim3(64), 0, s, ks);
        std::vector<unsigned long long> h((size_t)n * 16);
        (void)hipMemcpyAsync(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost, s);
        (void)hipStreamSynchronize(s);
        (void)hipFree(d);
        print_probe_stats("large stage", h, n);
      }
      return;
    }
    if (bw == 1 && big_slim(k) == BIG_SLIM_MINW) hipLaunchKernelGGL((cedar_probe_kernel<64, 1024, BIG_SLIM_MINW, false, 1, true, true>), dim3(n), dim3(64), 0, s, k);
    else if (bw == 1 && big_slim(k)) hipLaunchKernelGGL((cedar_probe_kernel<64, 1024, BIG_MINW, false, 1, true, true>), dim3(n), dim3(64), 0, s, k);
    else if (bw == 1) hipLaunchKernelGGL((cedar_probe_kernel<64, 1024, BIG_MINW, false, 1, true>), dim3(n), dim3(64), 0, s, k);
    else hipLaunchKernelGGL((cedar_probe_kernel<64, 1024, BIG_MINW, false, WAVES, true>), dim3((n + WAVES - 1) / WAVES), dim3(BLOCK), 0, s, k);
    return;
  }
  if (!big && k.scan && !probe_stats() && probe_seg() == 8 && probe_occ() == 3) {
    // register targets: the candidate pass at 4 waves per SIMD (128 VGPRs; split at 8 + 4 measured
    // 3.62e8 decisions/s on C3 against 3.42e8 unconstrained, profiles/r02/ab_split2); the scan at
    // 6 (80 VGPRs): as fast as at 8 with its LDS staging (4.61e8 vs 4.62e8, profiles/r02/ab_scan_lds)
    // and no register spills, whose scratch writes were 0.5 GB of the step's 2.2 GB L2-miss
    // traffic at 8 (profiles/r02/pmc_s3e)
    static const uint32_t socc = [] { const char* e = std::getenv("CEDARGPU_SCAN_OCC"); return e ? (uint32_t)std::atoi(e) : 6u; }();
    static const uint32_t cocc = [] { const char* e = std::getenv("CEDARGPU_CAND_OCC"); return e ? (uint32_t)std::atoi(e) : 4u; }();
    const dim3 sg((n + 7) / 8), sb(64);
    static const bool sstats = std::getenv("CEDARGPU_SCAN_STATS") != nullptr;
    if (k.req_idx) {  // a follow-up over the first pass's requests: their buckets are scanned
    } else if (sstats) {
      unsigned long long* d = nullptr;
      std::vector<unsigned long long> h(16, 0);
      if (hipMalloc((void**)&d, 16 * 8) == hipSuccess) {
        KArgs ks = k;
        ks.stats = d;
        (void)hipMemsetAsync(d, 0, 16 * 8, s);
        if (k.scan_filt && k.sbits_words) hipLaunchKernelGGL((cedar_scan_kernel<8, 6, true, true>), sg, sb, 0, s, ks);
        else hipLaunchKernelGGL((cedar_scan_kernel<8, 6, false, true>), sg, sb, 0, s, ks);
        (void)hipMemcpyAsync(h.data(), d, 16 * 8, hipMemcpyDeviceToHost, s);
        (void)hipStreamSynchronize(s);
        (void)hipFree(d);
        const double r = h[0] ? (double)h[0] : 1.0, w = (double)sg.x;
        std::fprintf(stderr,
                     "scan stats: requests %llu | per request: keys %.2f L1 probes %.2f found %.2f | L2 probes %.2f found %.2f | "
                     "per wave: iterations %.2f, segment-iterations %.2f (L2 %.2f) | cycles prologue %.0f loop %.0f | bitsets: "
                     "eligible %llu encoder-resolved %llu listed-path %llu, contexts found %.2f listed %.2f per request\n",
                     h[0], h[10] / r, h[1] / r, h[2] / r, h[3] / r, h[4] / r, h[5] / w, h[7] / w, h[6] / w, h[8] / w, h[9] / w,
                     h[15], h[13], h[11], h[12] / r, h[14] / r);
      }
    } else if (k.scan_filt && k.sbits_words) {
      static const bool lookup = std::getenv("CEDARGPU_SCAN_LOOKUP") && *std::getenv("CEDARGPU_SCAN_LOOKUP") == '1';
      if (lookup) hipLaunchKernelGGL((cedar_scan_kernel<8, 6, true, false, true>), sg, sb, 0, s, k);
      else if (socc == 6) hipLaunchKernelGGL((cedar_scan_kernel<8, 6, true>), sg, sb, 0, s, k);
      else if (socc == 7) hipLaunchKernelGGL((cedar_scan_kernel<8, 7, true>), sg, sb, 0, s, k);
      else if (socc == 8) hipLaunchKernelGGL((cedar_scan_kernel<8, 8, true>), sg, sb, 0, s, k);
      else hipLaunchKernelGGL((cedar_scan_kernel<8, 1, true>), sg, sb, 0, s, k);
    } else if (socc == 8) hipLaunchKernelGGL((cedar_scan_kernel<8, 8>), sg, sb, 0, s, k);
    else if (socc == 6) hipLaunchKernelGGL((cedar_scan_kernel<8, 6>), sg, sb, 0, s, k);
    else hipLaunchKernelGGL((cedar_scan_kernel<8>), sg, sb, 0, s, k);
    if (!k.req_idx) mark(PH_SCAN, s);
    static const bool cstats = std::getenv("CEDARGPU_CAND_STATS") != nullptr;
    if (cstats && !k.req_idx) {  // the candidate pass's work counters (profiling)
      const size_t nw = (n + 7) / 8;
      unsigned long long* d = nullptr;
      if (hipMalloc((void**)&d, (nw * 16 + 2) * 8) == hipSuccess) {
        KArgs ks = k;
        ks.stats = d;
        (void)hipMemsetAsync(d, 0, (nw * 16 + 2) * 8, s);
        hipLaunchKernelGGL((cedar_probe_kernel<8, 64, 4, true, 1, true>), dim3((n + 7) / 8), dim3(64), 0, s, ks);
        std::vector<unsigned long long> h(nw * 16 + 2);
        (void)hipMemcpyAsync(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost, s);
        (void)hipStreamSynchronize(s);
        (void)hipFree(d);
        print_probe_stats("candidate pass", h, nw);
        std::fprintf(stderr, "candidate sharing: %llu candidates, %llu of distinct buckets per wave round (distinct / total %.3f)\n",
                     h[nw * 16], h[nw * 16 + 1], h[nw * 16] ? (double)h[nw * 16 + 1] / (double)h[nw * 16] : 0.0);
      }
      return;
    }
    // The compact candidate pass (CEDARGPU_CAND_COMPACT=0: off): images whose hot values and like
    // words fit 16 entries take 32-hit rows and 16-entry hot rows, and spend the 4 KB of LDS that
    // saves on each lane's head atoms (SegLds::at4): 10.1 KB per wave as before, 4 waves per SIMD
    // (CEDARGPU_CAND_OCC=5: 96 VGPRs, which spills 128 B per lane: 0.99 vs 0.67 ms, gpurun_out/r05g)
    static const bool compact_on = !(std::getenv("CEDARGPU_CAND_COMPACT") && *std::getenv("CEDARGPU_CAND_COMPACT") == '0');
    const uint32_t hot_need = k.n_hot + (k.like_base != 0xFFFFFFFFu ? 3u * (uint32_t)__builtin_popcount(k.lslot) : 0u);
    static const uint32_t cocc_c = [] { const char* e = std::getenv("CEDARGPU_CAND_OCC"); return e ? (uint32_t)std::atoi(e) : 4u; }();
    if (compact_on && hot_need <= 16 && cocc_c == 4)
      hipLaunchKernelGGL((cedar_probe_kernel<8, 32, 4, false, 1, true, false, 16>), dim3((n + 7) / 8), dim3(64), 0, s, k);
    else if (cocc == 4) hipLaunchKernelGGL((cedar_probe_kernel<8, 64, 4, false, 1, true>), dim3((n + 7) / 8), dim3(64), 0, s, k);
    else hipLaunchKernelGGL((cedar_probe_kernel<8, 64, 3, false, 1, true>), dim3((n + 7) / 8), dim3(64), 0, s, k);
    return;
  }
  const uint32_t seg = big ? 64u : probe_seg();
  const bool w1 = (seg == 16 && (probe_occ() == 4 || probe_occ() == 5)) || (seg == 8 && (probe_occ() == 3 || probe_occ() == 4));
  const uint32_t wpb = (!big && w1 && !probe_stats()) ? probe_wpb() : WAVES;
  const uint32_t per_block = wpb * (64 / seg);
  const dim3 grid((n + per_block - 1) / per_block);
  const uint32_t occ = probe_occ();
  if (!big && probe_stats()) {
    const size_t nw = (size_t)grid.x * WAVES;
    unsigned long long* dstats = nullptr;
    if (hipMalloc((void**)&dstats, nw * 16 * sizeof(unsigned long long)) != hipSuccess) return;
    KArgs ks = k;
    ks.stats = dstats;
    std::vector<unsigned long long> h(nw * 16);
    (void)hipMemsetAsync(dstats, 0, h.size() * sizeof(unsigned long long), s);
    if (seg == 8) hipLaunchKernelGGL((cedar_probe_kernel<8, 64, 3, true>), grid, dim3(BLOCK), 0, s, ks);
    else hipLaunchKernelGGL((cedar_probe_kernel<16, 64, 4, true>), grid, dim3(BLOCK), 0, s, ks);
    (void)hipMemcpyAsync(h.data(), dstats, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost, s);
    (void)hipStreamSynchronize(s);
    (void)hipFree(dstats);
    print_probe_stats("probe", h, nw);
    return;
  }
  if (big) hipLaunchKernelGGL((cedar_probe_kernel<64, 1024>), grid, dim3(BLOCK), 0, s, k);
  else if (seg == 16 && occ == 4 && wpb == 1) hipLaunchKernelGGL((cedar_probe_kernel<16, 64, 4, false, 1>), grid, dim3(64), 0, s, k);
  else if (seg == 16 && occ == 4 && wpb == 2) hipLaunchKernelGGL((cedar_probe_kernel<16, 64, 4, false, 2>), grid, dim3(128), 0, s, k);
  else if (seg == 16 && occ == 4) hipLaunchKernelGGL((cedar_probe_kernel<16, 64, 4>), grid, dim3(BLOCK), 0, s, k);
  else if (seg == 16 && occ == 5 && wpb == 1) hipLaunchKernelGGL((cedar_probe_kernel<16, 64, 5, false, 1>), grid, dim3(64), 0, s, k);
  else if (seg == 16 && occ == 5) hipLaunchKernelGGL((cedar_probe_kernel<16, 64, 5>), grid, dim3(BLOCK), 0, s, k);
  else if (seg == 16) hipLaunchKernelGGL((cedar_probe_kernel<16, 64>), grid, dim3(BLOCK), 0, s, k);
  else if (seg == 8 && occ == 3 && wpb == 1) hipLaunchKernelGGL((cedar_probe_kernel<8, 64, 3, false, 1>), grid, dim3(64), 0, s, k);
  else if (seg == 8 && occ == 4 && wpb == 1) hipLaunchKernelGGL((cedar_probe_kernel<8, 64, 4, false, 1>), grid, dim3(64), 0, s, k);
  else if (seg == 8) hipLaunchKernelGGL((cedar_probe_kernel<8, 64, 3>), grid, dim3(BLOCK), 0, s, k);
  else if (seg == 32) hipLaunchKernelGGL((cedar_probe_kernel<32, 64>), grid, dim3(BLOCK), 0, s, k);
  else hipLaunchKernelGGL((cedar_probe_kernel<64, 64>), grid, dim3(BLOCK), 0, s, k);
}

// the policy-stream kernel for n requests: without bytecode, with it, or with it on the global
// lane area (an image whose bytecode needs more lane scratch than the private array holds)
static void launch_stream(const DevImage& img, const KArgs& k, uint32_t n, hipStream_t s) {
  auto kern = img.lane_need > LANE_WORDS ? cedar_eval_kernel<true, true>
              : img.has_bytecode          ? cedar_eval_kernel<true>
                                          : cedar_eval_kernel<false>;
  hipLaunchKernelGGL(kern, dim3((n + BLOCK - 1) / BLOCK), dim3(BLOCK), lds_bytes(img), s, k);
}

static void launch_eval(const DevImage& img, const KArgs& k, uint32_t n, hipStream_t s) {
  if (img.indexed)
    launch_probe(k, n, s);
  else
    launch_stream(img, k, n, s);
}

// One complete evaluation step of a batch, stream-ordered with no host round trip: the first
// pass over every request, then the gather of the requests it left unfinished and the three
// follow-up launches over them (their counts read on the device). dev_eval enqueues it once;
// dev_time_eval times it.
static int enqueue_step(const DevImage& img, DevBatch& b, hipStream_t s) {
  KArgs k = make_args(img, b, nullptr, b.n, b.res, b.reasons_f, b.reasons_p, b.errs, b.capr, b.cape);
  if (b.small) {
    // one launch: a wave per request probes the index itself (no scan lists), evaluates its
    // candidates and merges up to 1,024 hits; the reason capacity was sized for it at submit, and
    // a longer deciding list goes to an overflow slot (the FU_BIG worklist's entries, SLIM form)
    mark(PH_GROUP, s);
    const auto& f = b.fu[FU_BIG];
    if (b.fu_cnt && f.cap && big_slim(k)) {
      if (b.stepped) HIPCHK(hipMemsetAsync(b.fu_cnt, 0, (FU_KINDS + 1) * 4, s), "memset worklists");
      k.ovf_cnt = b.fu_cnt + FU_BIG;
      k.ovf_ids = f.ids; k.ovf_res = f.res; k.ovf_rf = f.rf; k.ovf_er = f.er;
      k.ovf_cap = f.cap; k.ovf_capr = f.capr; k.ovf_cape = f.cape;
    }
    b.stepped = true;
    if (big_slim(k)) hipLaunchKernelGGL((cedar_probe_kernel<64, 1024, BIG_SLIM_MINW, false, 1, false, true>), dim3(b.n), dim3(64), 0, s, k);
    else hipLaunchKernelGGL((cedar_probe_kernel<64, 1024, BIG_MINW, false, 1, false>), dim3(b.n), dim3(64), 0, s, k);
    HIPCHK(hipGetLastError(), "launch");
    for (uint32_t p = PH_SCAN; p < STEP_PHASES; p++) mark(p, s);
    return 0;
  }
  set_scan(k, b);
  // the candidate pass finishes long reason lists itself, into the long-list follow-up's worklist
  // (entries flagged FU_DONE: that launch skips them, the host folds them); CEDARGPU_LONG_SLOTS=0
  // leaves them to the follow-up launch
  static const bool long_slots = !(std::getenv("CEDARGPU_LONG_SLOTS") && *std::getenv("CEDARGPU_LONG_SLOTS") == '0');
  if (long_slots && b.fu_cnt && b.fu[FU_OVF].cap && img.indexed) {
    const auto& f = b.fu[FU_OVF];
    k.ovf_cnt = b.fu_cnt + FU_OVF;
    k.ovf_ids = f.ids; k.ovf_res = f.res; k.ovf_rf = f.rf; k.ovf_er = f.er;
    k.ovf_cap = f.cap; k.ovf_capr = f.capr; k.ovf_cape = f.cape;
  }
  if (b.ord) {  // grouped batch: this step's order and its rows in that order (group.hip)
    // (the worklist counters and the scan's bad-index count cleared by the grouping's first kernel)
    if (group_enqueue(b.gkeys, b.rows, b.n, b.row_words, b.grows, b.ord, b.gkeys2, b.gvals, b.grp_temp, b.grp_temp_bytes, s,
                      b.fu_cnt, b.fu_cnt ? FU_KINDS + 1 : 0u)) {
      g_err = "request grouping failed";
      return -4;
    }
  }
  mark(PH_GROUP, s);
  // the worklist counters and the scan's bad-index count start at zero before the first pass
  if (b.fu_cnt && !b.ord) HIPCHK(hipMemsetAsync(b.fu_cnt, 0, (FU_KINDS + 1) * 4, s), "memset worklists");
  const bool two = img.indexed && split_on() && !probe_stats() && probe_seg() == 8 && probe_occ() == 3;
  launch_eval(img, k, b.n, s);
  HIPCHK(hipGetLastError(), "launch");
  if (!two) mark(PH_SCAN, s);  // a one-kernel first pass: all of it in the scan phase
  mark(PH_CAND, s);
  if (!b.fu_cnt) {
    for (uint32_t p = PH_GATHER; p < STEP_PHASES; p++) mark(p, s);
    return 0;
  }
  FuLists wl;
  for (uint32_t q = 0; q < FU_KINDS; q++) { wl.ids[q] = b.fu[q].ids; wl.cap[q] = b.fu[q].cap; }
  hipLaunchKernelGGL(cedar_fu_gather, dim3((b.n + GATHER_ITEMS * 256 - 1) / (GATHER_ITEMS * 256)), dim3(256), 0, s, b.res,
                     b.n, img.indexed, b.fu_cnt, wl, (const uint32_t*)b.ord, b.ord ? b.pos_of : nullptr);
  mark(PH_GATHER, s);
  for (uint32_t q = 0; q < FU_KINDS; q++) {
    const auto& f = b.fu[q];
    if (f.cap) {
      KArgs fk = make_args(img, b, f.ids, f.cap, f.res, f.rf, f.rp, f.er, f.capr, f.cape);
      fk.n_dev = b.fu_cnt + q;
      set_scan(fk, b);  // the probe-kernel follow-ups read the first pass's buckets
      // (long lists too run on the large stage: it reads its request's pairs out of the wave's
      // list; the pooled candidate pass reads whole lists of first-pass waves only)
      if (q == FU_GEN) launch_stream(img, fk, f.cap, s);
      else launch_probe(fk, f.cap, s, true);
    }
    mark(PH_FU_BIG + q, s);
  }
  HIPCHK(hipGetLastError(), "launch follow-up");
  return 0;
}

int dev_eval(const DevImage& img, DevBatch& b, void* stream) {
  HIPCHK(hipSetDevice(b.device), "hipSetDevice");
  if (b.n == 0) return 0;
  if (img.device != b.device) { g_err = "image and batch live on different devices"; return -2; }
  return enqueue_step(img, b, (hipStream_t)stream);
}

// Re-evaluates a subset of requests (overflowed result lists) with larger capacities; results are
// compact in subset order. _begin enqueues (H2D of the indices, launch, D2H) on `stream` without
// waiting, so several subsets share one host round trip; _end waits and points at the results in
// the job's pinned block; _release returns the job's blocks to the pool.
int dev_subset_begin(const DevImage& img, const DevBatch& b, const uint32_t* idx, uint32_t n, uint32_t capr,
                     uint32_t cape, int probe, void* stream, DevSubset* job) {
  HIPCHK(hipSetDevice(b.device), "hipSetDevice");
  hipStream_t s = (hipStream_t)stream;
  *job = DevSubset();
  if (n == 0) return 0;
  if (!b.pool) { g_err = "batch has no buffer pool"; return -4; }
  for (uint32_t i = 0; i < n; i++) if (idx[i] >= b.n) { g_err = "request index out of range"; return -2; }
  if (n > b.n && img.lane_need > LANE_WORDS) { g_err = "subset larger than its batch's lane area"; return -2; }
  // one device block [idx | res | reasons_f | reasons_p | errs] and one pinned block, from the pool
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  DevSubset j;
  j.pool = b.pool;
  j.stream = stream;
  j.n = n;
  j.capr = capr;
  j.cape = cape;
  j.o_res = al((size_t)n * 4);
  j.o_rf = j.o_res + al((size_t)n * 2 * 4);
  const bool one_list = probe && img.indexed;  // the probe kernel writes only the deciding list
  j.o_rp = one_list ? j.o_rf : j.o_rf + al((size_t)n * capr * 4);
  j.o_er = j.o_rp + al((size_t)n * capr * 4);
  j.total = j.o_er + al((size_t)n * cape * ERR_WORDS * 4);
  int rc;
  if ((rc = pool_get(b.pool, false, j.total, &j.dblk, &j.dcls))) return rc;
  if ((rc = pool_get(b.pool, true, j.total, &j.hblk, &j.hcls))) { pool_put(b.pool, false, j.dblk, j.dcls); return rc; }
  uint8_t* d8 = (uint8_t*)j.dblk;
  uint8_t* h8 = (uint8_t*)j.hblk;
  std::memcpy(h8, idx, (size_t)n * 4);
  *job = j;  // blocks owned by the job from here on (returned by dev_subset_release)
  hipError_t e;
  hipEvent_t ev;
  if ((e = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess) return fail(e, "event");
  job->done = (void*)ev;
  if ((e = hipMemcpyAsync(d8, h8, (size_t)n * 4, hipMemcpyHostToDevice, s)) != hipSuccess) return fail(e, "H2D");
  KArgs k = make_args(img, b, (uint32_t*)d8, n, (uint32_t*)(d8 + j.o_res), (uint32_t*)(d8 + j.o_rf),
                      (uint32_t*)(d8 + j.o_rp), (uint32_t*)(d8 + j.o_er), capr, cape);
  if (probe && img.indexed)
    launch_probe(k, n, s, probe == 2);
  else
    launch_stream(img, k, n, s);
  if ((e = hipGetLastError()) != hipSuccess) return fail(e, "launch");
  if ((e = hipMemcpyAsync(h8 + j.o_res, d8 + j.o_res, j.total - j.o_res, hipMemcpyDeviceToHost, s)) != hipSuccess) return fail(e, "D2H");
  if ((e = hipEventRecord(ev, s)) != hipSuccess) return fail(e, "event record");
  return 0;
}

int64_t dev_now_ns() {
  return (int64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Waits for `ev` until deadline_ns (< 0: none): spins with yields for the first ~500 us (results
// of a latency-bound batch arrive within that: the serving queue's submitter polls every batch in
// 10 ms slices), then sleeps 10 us between queries.
// t0 (0: now) is when the caller's first wait on this event began: a caller that waits in slices
// spins once per event, not once per slice.
static int wait_event(hipEvent_t ev, int64_t deadline_ns, const char* what, int64_t t0 = 0) {
  if (deadline_ns < 0) {
    HIPCHK(hipEventSynchronize(ev), what);
    return 0;
  }
  if (!t0) t0 = dev_now_ns();
  for (;;) {
    const hipError_t q = hipEventQuery(ev);
    if (q == hipSuccess) return 0;
    if (q != hipErrorNotReady) return fail(q, what);
    const int64_t now = dev_now_ns();
    if (now >= deadline_ns) {
      g_err = std::string(what) + ": deadline exceeded";
      return DEV_TIMEOUT;
    }
    if (now - t0 < 500000) std::this_thread::yield();
    else std::this_thread::sleep_for(std::chrono::microseconds(10));
  }
}

int dev_subset_end(DevSubset* job, SubsetView* v, int64_t deadline_ns) {
  *v = SubsetView();
  if (!job->dblk) return 0;
  const int rc = wait_event((hipEvent_t)job->done, deadline_ns, "re-run");
  if (rc == DEV_TIMEOUT) return rc;  // still in flight: the caller keeps the job until the stream drains
  if (rc) {
    (void)hipStreamSynchronize((hipStream_t)job->stream);  // nothing of ours in flight before release
    dev_subset_release(job);
    return rc;
  }
  const uint8_t* h8 = (const uint8_t*)job->hblk;
  v->res = (const uint32_t*)(h8 + job->o_res);
  v->rf = (const uint32_t*)(h8 + job->o_rf);
  v->rp = (const uint32_t*)(h8 + job->o_rp);
  v->er = (const uint32_t*)(h8 + job->o_er);
  return 0;
}

void dev_subset_release(DevSubset* job) {
  if (job->done) (void)hipEventDestroy((hipEvent_t)job->done);
  if (job->pool) {
    pool_put(job->pool, false, job->dblk, job->dcls);
    pool_put(job->pool, true, job->hblk, job->hcls);
  }
  *job = DevSubset();
}

// Points the host batch's result arrays into the pinned staging block the results were copied to
// (the block stays with the batch until dev_batch_free).
static void bind_results(const DevBatch& b, Batch& host) {
  host.capr = b.capr;
  host.cape = b.cape;
  // (zero-copy: the results sit at zc_out, whose device view is the one the kernel wrote through)
  uint8_t* st = b.zc ? b.zc_out : (uint8_t*)b.stage;
  const uint8_t* base = b.zc ? (const uint8_t*)b.res : (const uint8_t*)b.out_blk;
  auto at = [&](const uint32_t* dev) { return (uint32_t*)(st + ((const uint8_t*)dev - base)); };
  host.res = b.n ? at(b.res) : nullptr;
  host.reasons_f = b.n ? at(b.reasons_f) : nullptr;
  host.reasons_p = b.n ? at(b.reasons_p) : nullptr;
  host.errs = b.n ? at(b.errs) : nullptr;
  host.pos_of = (b.n && b.pos_of) ? at(b.pos_of) : nullptr;
  host.fu_cnt = (b.n && b.fu_cnt) ? (b.zc ? b.zc_cnt : at(b.fu_cnt)) : nullptr;
  for (uint32_t k = 0; k < FU_KINDS; k++) {
    host.fu[k] = Batch::FollowUp();
    const auto& f = b.fu[k];
    if (!b.n || !f.cap) continue;
    host.fu[k].ids = at(f.ids);
    host.fu[k].res = at(f.res);
    host.fu[k].rf = at(f.rf);
    host.fu[k].rp = at(f.rp);
    host.fu[k].er = at(f.er);
    host.fu[k].cap = f.cap;
    host.fu[k].capr = f.capr;
    host.fu[k].cape = f.cape;
  }
}

// A small batch's overflow slots after its results arrived: the ones it took (the counter), each
// array's used prefix (the kernel has finished: plain copies, off the batch's stream, which may
// already run the next batch).
static int fetch_overflow(DevBatch& b) {
  if (b.zc || !b.dl_bytes || b.dl_bytes >= b.out_bytes || !b.fu_cnt) return 0;
  const uint8_t* base = (const uint8_t*)b.out_blk;
  uint8_t* st = (uint8_t*)b.stage;
  const uint32_t taken = *(const uint32_t*)(st + ((const uint8_t*)(b.fu_cnt + FU_BIG) - base));
  const auto& f = b.fu[FU_BIG];
  const size_t used = std::min<uint32_t>(taken, f.cap);
  if (!used) return 0;
  const std::pair<const uint32_t*, size_t> arr[4] = {
      {f.ids, used * 4}, {f.res, used * 8}, {f.rf, used * f.capr * 4}, {f.er, used * f.cape * ERR_WORDS * 4}};
  // (four copies on the null stream, one wait: the batch's own stream may already run the next
  // batch, and the null stream does not order against these non-blocking streams)
  for (const auto& a : arr) {
    const size_t o = (const uint8_t*)a.first - base;
    HIPCHK(hipMemcpyAsync(st + o, base + o, a.second, hipMemcpyDeviceToHost, nullptr), "D2H overflow slots");
  }
  HIPCHK(hipStreamSynchronize(nullptr), "D2H overflow slots");
  return 0;
}

int dev_download(DevBatch& b, Batch& host, void* stream) {
  HIPCHK(hipSetDevice(b.device), "hipSetDevice");
  hipStream_t s = (hipStream_t)stream;
  if (b.zc && b.fu_cnt) HIPCHK(hipMemcpyAsync(b.zc_cnt, b.fu_cnt, (FU_KINDS + 1) * 4, hipMemcpyDeviceToHost, s), "D2H counters");
  else if (b.n) HIPCHK(hipMemcpyAsync(b.stage, b.out_blk, b.dl_bytes ? b.dl_bytes : b.out_bytes, hipMemcpyDeviceToHost, s), "D2H results");
  HIPCHK(hipStreamSynchronize(s), "sync download");
  b.pending = false;
  if (const int rc = fetch_overflow(b)) return rc;
  bind_results(b, host);
  return 0;
}

int dev_download_async(DevBatch& b, void* stream) {
  HIPCHK(hipSetDevice(b.device), "hipSetDevice");
  hipStream_t s = (hipStream_t)stream;
  if (!b.done) {
    hipEvent_t e;
    HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming), "event");
    b.done = (void*)e;
  }
  if (b.pev[2]) HIPCHK(hipEventRecord((hipEvent_t)b.pev[2], s), "event record");
  if (b.zc && b.fu_cnt) HIPCHK(hipMemcpyAsync(b.zc_cnt, b.fu_cnt, (FU_KINDS + 1) * 4, hipMemcpyDeviceToHost, s), "D2H counters");
  else if (b.n) HIPCHK(hipMemcpyAsync(b.stage, b.out_blk, b.dl_bytes ? b.dl_bytes : b.out_bytes, hipMemcpyDeviceToHost, s), "D2H results");
  if (b.pev[3]) HIPCHK(hipEventRecord((hipEvent_t)b.pev[3], s), "event record");
  HIPCHK(hipEventRecord((hipEvent_t)b.done, s), "event record");
  b.wait_t0 = 0;
  return 0;
}



int dev_download_finish(DevBatch& b, Batch& host, int64_t deadline_ns) {
  HIPCHK(hipSetDevice(b.device), "hipSetDevice");
  if (b.done) {
    if (!b.wait_t0) b.wait_t0 = dev_now_ns();
    const int rc = wait_event((hipEvent_t)b.done, deadline_ns, "batch", b.wait_t0);
    if (rc) return rc;  // DEV_TIMEOUT: still in flight (pending), wait again or destroy
  }
  b.pending = false;
  if (const int rc = fetch_overflow(b)) return rc;
  bind_results(b, host);
  return 0;
}

// A one-thread kernel that waits on the device wall clock (wall_clock64, constant rate `khz`).
__global__ void __launch_bounds__(64) cedar_stall_kernel(uint64_t ticks) {
  if (threadIdx.x != 0) return;
  const uint64_t t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
}

int dev_stall(int device, void* stream, uint64_t us) {
  HIPCHK(hipSetDevice(device), "hipSetDevice");
  int khz = 0;
  HIPCHK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device), "wall clock rate");
  const uint64_t ticks = std::min<uint64_t>(us, 2000000u) * (uint64_t)std::max(khz, 1) / 1000u;
  hipLaunchKernelGGL(cedar_stall_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, ticks);
  HIPCHK(hipGetLastError(), "launch stall");
  return 0;
}

int dev_time_split(const DevImage& img, DevBatch& b, uint32_t iters, void* stream, float* ms_phase, float* ms_total) {
  HIPCHK(hipSetDevice(b.device), "hipSetDevice");
  hipStream_t s = (hipStream_t)stream;
  // every event created is destroyed on every path (and the step's marks never outlive them)
  struct Events {
    std::vector<hipEvent_t> v;
    ~Events() {
      t_marks = nullptr;
      for (auto e : v) (void)hipEventDestroy(e);
    }
  } ev;
  ev.v.reserve((size_t)iters * (STEP_PHASES + 1));
  for (size_t i = 0; i < (size_t)iters * (STEP_PHASES + 1); i++) {
    hipEvent_t e;
    HIPCHK(hipEventCreate(&e), "event");
    ev.v.push_back(e);
  }
  for (uint32_t i = 0; i < iters; i++) {
    t_marks = &ev.v[(size_t)i * (STEP_PHASES + 1)];
    HIPCHK(hipEventRecord(t_marks[0], s), "event record");
    const int rc = enqueue_step(img, b, s);
    t_marks = nullptr;
    if (rc) return rc;
  }
  HIPCHK(hipEventSynchronize(ev.v.back()), "event sync");
  for (uint32_t p = 0; p < STEP_PHASES; p++) ms_phase[p] = 0.f;
  *ms_total = 0.f;
  // enqueue_step marks every phase of every step (an empty phase is two adjacent marks): a phase
  // without its events is an error, not a zero
  for (uint32_t i = 0; i < iters; i++) {
    const hipEvent_t* m = &ev.v[(size_t)i * (STEP_PHASES + 1)];
    for (uint32_t p = 0; p < STEP_PHASES; p++) {
      float t = 0.f;
      HIPCHK(hipEventElapsedTime(&t, m[p], m[p + 1]), "phase elapsed time");
      ms_phase[p] += t;
    }
    float t = 0.f;
    HIPCHK(hipEventElapsedTime(&t, m[0], m[STEP_PHASES]), "step elapsed time");
    *ms_total += t;
  }
  return 0;
}

int dev_time_eval(const DevImage& img, DevBatch& b, uint32_t iters, void* stream, float* ms_total) {
  HIPCHK(hipSetDevice(b.device), "hipSetDevice");
  hipStream_t s = (hipStream_t)stream;
  struct Ev {
    hipEvent_t e = nullptr;
    ~Ev() { if (e) (void)hipEventDestroy(e); }
  } e0, e1;
  HIPCHK(hipEventCreate(&e0.e), "event");
  HIPCHK(hipEventCreate(&e1.e), "event");
  HIPCHK(hipEventRecord(e0.e, s), "event record");
  for (uint32_t i = 0; i < iters; i++) {
    const int rc = enqueue_step(img, b, s);
    if (rc) return rc;
  }
  HIPCHK(hipEventRecord(e1.e, s), "event record");
  HIPCHK(hipEventSynchronize(e1.e), "event sync");
  HIPCHK(hipEventElapsedTime(ms_total, e0.e, e1.e), "elapsed");
  return 0;
}

}  // namespace cg
