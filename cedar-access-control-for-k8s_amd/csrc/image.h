// Compiled policy image + request batch layout shared by the host compiler/encoder and the
// gfx950 evaluation kernel. Plain integers only; included from both C++ and HIP.
//
// Layout in HBM (all u32 words unless noted)
// ------------------------------------------
// Image (replicated per GPU, read-only, uploaded once per policy epoch):
//   pol[n_pol * POL_WORDS]   policy descriptors, in tier order (scope + code range + effect)
//   tier_end[n_tiers]        exclusive end index of each tier in `pol`
//   code[]                   condition bytecode, 2 words per instruction
//   cpool[]                  constant pool (sets, records, patterns, scope action lists)
//   gstr_off[n_gstr + 1]     byte offsets of the global (policy) string table
//   gstr_bytes[]             string bytes
// Batch (per submission):
//   rows[R * row_words]      columnar request row: P/A/R UIDs, ancestor-list offsets and the
//                            image's hot attribute paths pre-resolved on the host (see RowW)
//   req_base[R]              word offset of request r's heap block in `heap`
//   heap[]                   per-request blocks: header, entity table, attribute data
//   bstr_off[n_bstr + 1], bstr_bytes[]  batch-local strings (ids >= n_gstr)
//   res[R * 2], reasons_f/p[R * capr], errs[R * cape * ERR_WORDS]   results
#pragma once
#include <stdint.h>

#if !defined(__HIPCC__) && !defined(__host__)
#define __host__
#define __device__
#endif

namespace cgi {

// ---- value encoding (memory form: 2 words) --------------------------------------------------
// w0 = tag << 28 | x (28 bits), w1 = y
enum Tag : uint32_t {
  T_NONE = 0,
  T_BOOL = 1,    // y = 0/1
  T_LONG = 2,    // memory: y = int32 value (sign-extended); register form: y = lo, z = hi
  T_LONGREF = 3, // memory only: x = ref -> [lo, hi]
  T_STR = 4,     // y = string id
  T_ENT = 5,     // x = type string id, y = id string id
  T_SET = 6,     // x = ref -> [n, (w0, w1) * n]
  T_REC = 7,     // x = ref -> [n, (key, w0, w1) * n] sorted by key id
  T_DEC = 8,     // x = ref -> [lo, hi]
  T_IP = 9,      // x = ref -> [v6 | prefix << 8, a0, a1, a2, a3] (big-endian address bytes)
};
constexpr uint32_t TAG_SHIFT = 28;
constexpr uint32_t X_MASK = 0x0FFFFFFFu;
// refs: space (2 bits) | word offset (26 bits). Heap refs are relative to the request block.
constexpr uint32_t SPACE_SHIFT = 26;
constexpr uint32_t OFF_MASK = 0x03FFFFFFu;
enum Space : uint32_t { SP_HEAP = 0, SP_CPOOL = 1, SP_LANE = 2 };

__host__ __device__ constexpr inline uint32_t mk_w0(uint32_t tag, uint32_t x) { return (tag << TAG_SHIFT) | (x & X_MASK); }
__host__ __device__ constexpr inline uint32_t mk_ref(uint32_t space, uint32_t off) { return (space << SPACE_SHIFT) | (off & OFF_MASK); }

// ---- request block header -------------------------------------------------------------------
// (the principal / action / resource UIDs are the row's RW_P / RW_A / RW_R: every kernel reads the
// row before the block, so the block does not repeat them)
enum ReqHdr : uint32_t {
  RH_NENT = 0,
  RH_CTX = 1,    // context value (REC, 2 words)
  RH_PIDX = 3,   // entity-table index of principal / action / resource (NO_ENT if absent)
  RH_AIDX = 4,
  RH_RIDX = 5,
  RH_SBASE = 6,  // index of the request's first string in the batch string table (bstr_off)
  RH_SCTX = 7,   // the request's scope contexts, resolved by the encoder (CTXR_SLOTS words, below)
  RH_WORDS = 11, // entity table follows: n_ent * ENT_WORDS
};
// Host-resolved scope contexts (image.h "scope bitsets"). A request's contexts depend on its
// action, resource and hot values only, never on its principal, so the encoder looks them up in
// the image's context table (Image::sctx, the host keeps a copy) exactly as cedar_scan_kernel
// would, and writes the ones it finds into RH_SCTX: combo | bitset row << CTXR_ROW each, CTXR_EMPTY
// after the last. The row's RW_ASELF carries ASELF_CTXR when it did (the scan then skips the
// context filter, the table probes and the list-slot reads they need); when the request's
// contexts are more than CTX_CAP or it finds more than CTXR_SLOTS, the scan looks them up itself.
constexpr uint32_t CTXR_SLOTS = 4, CTXR_EMPTY = 0xFFFFFFFFu, CTXR_ROW = 5, CTX_CAP = 16;
enum EntRow : uint32_t { ER_TYPE = 0, ER_ID = 1, ER_ATTR0 = 2, ER_ATTR1 = 3, ER_ANC = 4, ER_PAD = 5, ENT_WORDS = 6 };
constexpr uint32_t NO_ENT = 0xFFFFFFFFu;
// Ancestor lists of request entities live outside their blocks: the batch heap holds each distinct
// list once ([n, (type, id) x n], then the key-entity indices on a scope-bitset image), ahead of the
// first block that uses it, and every block whose entity has that ancestry points back at it. So a
// table entity's ER_ANC is an SP_HEAP ref whose 26-bit offset is signed (two's complement,
// block-relative, at most ANC_REACH words back), and the row's RW_PANC / RW_RANC / RW_AANC are
// signed 32-bit block-relative offsets of the first pair.
constexpr uint32_t ANC_REACH = (1u << 25) - 1;
__host__ __device__ constexpr inline int32_t sext26(uint32_t off) { return (int32_t)(off << 6) >> 6; }

// ---- static entities (the image's entity hierarchy) -------------------------------------------
// Entities compiled into the image (cg_compiler_set_entities): a group / namespace hierarchy the
// requests' EntityMaps do not carry. Evaluation sees each request's EntityMap merged with them: a
// static entity the request lacks is present; for a UID in both, the request's attributes and the
// union of both parent lists. Device form: `srows` rows of ENT_WORDS laid out like the request
// entity table, with ER_ATTR* a record and ER_ANC a reference into the constant pool
// ([n, (type, id) x n]: the entity's transitive ancestors over the static edges, the compiled
// `in`-closure row); `shash` an open-addressed table of SH_WORDS slots [type, id, row + 1, 0].
// An entity index with ENT_STATIC set names static row (index & ~ENT_STATIC).
constexpr uint32_t ENT_STATIC = 0x40000000u, SH_WORDS = 4;
__host__ __device__ constexpr inline uint32_t uid_hash(uint32_t t, uint32_t i) {
  uint32_t h = (t * 0x9E3779B1u) ^ (i * 0x85EBCA77u);
  h ^= h >> 15;
  h *= 0x2C1B3C6Du;
  h ^= h >> 12;
  return h;
}

// ---- policy descriptor ----------------------------------------------------------------------
enum ScopeK : uint32_t { SK_ANY = 0, SK_EQ = 1, SK_IN = 2, SK_IS = 3, SK_ISIN = 4, SK_INSET = 5 };
enum PolFlags : uint32_t { PF_FORBID = 1, PF_ATOMIC = 2 };
enum PolW : uint32_t {
  PW_FLAGS = 0,   // bit0 forbid, bit1 atomic (code = atoms), bits 8..15 tier,
                  // bits 16..22 principal-entity bloom bit, bits 24..30 resource-entity bloom bit
  PW_KINDS = 1,   // p_kind | a_kind << 8 | r_kind << 16
  PW_P_TYPE = 2,  // is-type (string id)
  PW_P_ET = 3,    // entity type (string id)
  PW_P_EI = 4,    // entity id (string id)
  PW_A_ET = 5,    // eq/in: entity type; inset: count
  PW_A_EI = 6,    // eq/in: entity id;   inset: cpool offset of (type, id) pairs
  PW_R_TYPE = 7,
  PW_R_ET = 8,
  PW_R_EI = 9,
  PW_CODE = 10,   // pol[]: code word offset; stream records: global policy index (code follows)
  PW_CODE_N = 11, // code words
  PW_SLOTS = 12,  // bytecode: max register slot used + 1; atomic: words of atoms (data follows)
  PW_LANE = 13,   // bytecode: lane-scratch words needed; index heads: PW_EXT (full record offset)
  PW_AMASK0 = 14, // action scope as a mask over the image action table (valid when n_act <= 64)
  PW_AMASK1 = 15,
  POL_WORDS = 16,
};
constexpr uint32_t PW_EXT = PW_LANE;

// ---- scope index (probe kernel) ---------------------------------------------------------------
// Every policy of an all-atomic image is filed under keys that any request it can apply to (or
// error on) must enumerate:
//   level 1  a (principal, action, resource) triple; each component is the scope's entity (==,
//            in, is-in: the request enumerates its ancestor-or-self UIDs), its type (`is`), or a
//            wildcard; `action in [..]` files one key per listed action. The component kinds form
//            the key's combo (KC_*); the image records the combos in use (combo_mask) and a
//            request probes each used combo's product of its own candidate components;
//   level 2  the level-1 key plus (h, value): the constant c of an equality atom hot(h) == c that
//            every satisfying evaluation passes and that no erroring atom precedes; filed under
//            value c, and also under MISSING_W0 when an absent h would make that atom raise (no
//            `has h` guard before it).
// A request probes level 1 for its keys, then level 2 under each found key for every hot slot in
// the entry's hmask, with its own value of that slot (or MISSING_W0).
// btab (device): open addressing, linear probing, power-of-two slots of BT_WORDS, built at load
// from the blob's compact entry list (Image::btab, Image::btab_slots) by inserting each entry at
// its key's hash (l1: key_hash; l2: bucket_hash2 of it); slot layout:
//   [BT_USED | combo << 16 | (BT_L2 | h for level 2), p type, p id, a type, a id, r type, r id,
//    value w0 (level 1: cmask), value w1, first, count, hmask (level 1), l2 bloom x 4 (level 1)];
//   empty: word0 == 0.
//   The level-1 entry's 128-bit bloom (l2_bloom_bits) holds its level-2 keys: a request probes
//   level 2 only for (h, value) pairs it admits.
// Records: bstream[first * HEAD_WORDS ...] fixed heads (descriptor + the first 4 atoms) in bucket
// order; the head's PW_EXT is the absolute bstream offset of the full variable-length record
// (descriptor, atoms, atom data) in the ext area, which record-relative offsets address.
// Duplicate classes: policies whose records agree word for word (global index aside) are filed
// once, under the lowest-index member; its head's PW_CODE_N holds the bstream offset of the class
// list [n, member global indices ascending] (0: a policy alone), and a hit records every member.
constexpr uint32_t KC_WILD = 0, KC_ENT = 1, KC_TYPE = 2;  // component kinds
__host__ __device__ constexpr inline uint32_t key_combo(uint32_t pk, uint32_t ak, uint32_t rk) { return pk | (ak << 2) | (rk << 3); }
constexpr uint32_t KW_ANY = 0xFFFFFFFFu;  // id of a type-only component; both words of a wildcard
constexpr uint32_t BT_WORDS = 16, BT_USED = 0x80000000u, BT_L2 = 0x100, HEAD_WORDS = 32, HEAD_ATOMS = 4;
// key_hash = key_fin(key_pre(combo, action, resource), principal): the principal component is
// mixed last, so a request hashes the (combo, action, resource) prefix once per combo and each of
// its ~30 principal key ancestors in two multiply steps and a finalizer (cedar_scan_kernel).
__host__ __device__ constexpr inline uint32_t key_pre(uint32_t combo, uint32_t at, uint32_t ai, uint32_t rt, uint32_t ri) {
  uint32_t h = (combo + 1) * 0x9E3779B1u;
  h = (h ^ at) * 0x85EBCA77u; h = (h ^ ai) * 0xC2B2AE3Du;
  h = (h ^ rt) * 0x27D4EB2Fu; h = (h ^ ri) * 0x165667B1u;
  return h;
}
__host__ __device__ constexpr inline uint32_t key_fin(uint32_t pre, uint32_t pt, uint32_t pi) {
  uint32_t h = (pre ^ pt) * 0xD3A2646Du;
  h = (h ^ pi) * 0xFD7046C5u;
  h ^= h >> 16;
  h *= 0x7FEB352Du;
  h ^= h >> 15;
  return h;
}
__host__ __device__ constexpr inline uint32_t key_hash(uint32_t combo, uint32_t pt, uint32_t pi, uint32_t at, uint32_t ai,
                                                       uint32_t rt, uint32_t ri) {
  return key_fin(key_pre(combo, at, ai, rt, ri), pt, pi);
}
__host__ __device__ constexpr inline uint32_t bucket_hash2(uint32_t l1, uint32_t hslot, uint32_t v0, uint32_t v1) {
  uint32_t h = l1 ^ ((hslot + 1) * 0x27D4EB2Fu) ^ (v0 * 0x165667B1u) ^ (v1 * 0xD3A2646Cu);
  h ^= h >> 15;
  h *= 0x2C1B3C6Du;
  h ^= h >> 12;
  return h;
}

__host__ __device__ constexpr inline uint32_t l2_bloom_bits(uint32_t h2) {  // three 7-bit positions
  const uint32_t y = (h2 ^ (h2 >> 13)) * 0x5BD1E995u;
  return (y >> 11) & 0x1FFFFFu;
}
// Key filter of the scope index (bfilt): a blocked Bloom filter over the level-1 and level-2 key
// hashes, 3 bits in one 64-bit block (two words) per key, about 16 bits per entry: a few hundred KB
// that stay in L2. The block is the hash's low bits (h & fmask); the bit positions come from the
// top of h * φ, so a test costs one multiply beyond the key hash.
__host__ __device__ constexpr inline uint32_t filt_bits(uint32_t h) {  // b0 | b1 << 6 | b2 << 12
  const uint32_t y = h * 0x9E3779B1u;
  return (y >> 26) | (((y >> 20) & 63u) << 6) | (((y >> 14) & 63u) << 12);
}
__host__ __device__ constexpr inline uint64_t filt_need(uint32_t h) {  // the 3 bits as a 64-bit mask
  const uint32_t b = filt_bits(h);
  return (1ull << (b & 63u)) | (1ull << ((b >> 6) & 63u)) | (1ull << ((b >> 12) & 63u));
}

// Scope bitsets: exact membership tests for the scope-index keys whose principal component is an
// entity (combo with pkc == KC_ENT), at both levels. A key splits into its context and its
// principal key entity:
//   level 1: context (combo, action component, resource component, SCTX_L1, 0, 0); the bit is set
//            when the level-1 key files policies directly (an entry that only carries level-2 keys
//            has no bit: it decides nothing by itself);
//   level 2: context (combo, action, resource, hot slot h (| BT_CKEY for list keys), v0, v1); the
//            bit is set when that level-2 key exists.
// Each context in use has a row of sbits_words words, one bit per key entity (index into
// Image::key_ents, "kidx"), stored as (bits, rank) word pairs: rank = the set bits of every earlier
// word of every row, so a set bit's global rank is rank + popcount of the word's lower bits. svals
// holds each set bit's bucket at its rank, SVAL_WORDS each: (first head, head count) of the key's
// own scope-index entry, what a probe of that key in btab would return, and the bucket's presence
// mask (below). sctx: an open-addressed table of S slots (S
// a power of two) at ctx_key(key_pre(combo, at, ai, rt, ri), hs, v0, v1) & (S - 1), SCTX_WORDS
// each: [SCTX_USED | combo << 16 | hs, at, ai, rt, ri, v0, v1, row] (0 = empty; 32 bytes, one
// round trip, compared whole). A request looks up its contexts (per entity-principal combo: level
// 1, each value slot of l2_vmask with its own value, each element of its list slots in l2_lmask)
// and tests one bit per principal key ancestor in each context found (the encoder lists their kidx
// after the ancestor pairs: [n, (type, id) x n, kidx(self), kidx x keys], kidx ~0 for a UID that is
// no key entity); every set bit is a found bucket, read from svals at its rank: no key hash and no
// btab probe. On C3 that is ~8 bucket reads from a ~0.1 MB table per request instead of ~62
// level-1 probes of 64-byte slots and their level-2 follow-ups; the grouped requests of a wave
// share the rows. Images whose bitsets would exceed SBITS_MAX_BYTES have none (sbits_words == 0).
// Presence masks: a policy whose entry spine reaches `hot(h) has` (a single-level slot, so the
// test cannot raise) with its false edge UNSAT, before any atom that can raise, is UNSAT on every
// request without that attribute. A bucket's mask is the AND of its policies' such slots (in a
// bucket of a level-2 key's value, where the key atom cannot raise, also the `has` atoms after the
// key atom; slots 0..ASELF_PRES_SLOTS - 1 only); the scan lists a bucket from svals only when the
// request has every slot of its mask (the encoder's presence bits in the row's RW_ASELF), so such a
// request's candidates never include it.
// (Only the bitset path filters: a bucket reached by a btab probe is evaluated as before, which is
// the same answer.)
// Equality filters: in a bucket of a level-2 key's value, a policy whose spine after the key atom
// reaches `hot(h) == c` (c a string, Boolean or entity) with only atoms that cannot raise before
// it is UNSAT on every request whose slot h holds a value other than c. When every policy of the
// bucket has the same such (h, c), the bucket carries EQF_ON | h << EQF_SLOT_SHIFT | eqf_hash(c),
// and the scan skips it for a request whose hot value h is present (a missing or erroneous value
// makes the atom raise: the bucket stays) with another hash (equal values hash alike).
constexpr uint32_t EQF_ON = 0x80000000u, EQF_SLOT_SHIFT = 26, EQF_SLOTS = 16, EQF_HASH = (1u << EQF_SLOT_SHIFT) - 1u;
__host__ __device__ constexpr inline uint32_t eqf_hash(uint32_t w0, uint32_t w1) {
  // (the words prim_eq compares: an entity's type and id, another value's tag and word 1)
  const uint32_t a = (w0 >> TAG_SHIFT) == T_ENT ? w0 : (w0 >> TAG_SHIFT) << TAG_SHIFT;
  uint32_t h = (a * 0x9E3779B1u) ^ ((w1 + 0x7F4A7C15u) * 0x85EBCA77u);
  h ^= h >> 15;
  h *= 0x2C1B3C6Du;
  h ^= h >> 12;
  return h & EQF_HASH;
}
constexpr uint32_t SVAL_WORDS = 4;  // (first head, head count, presence mask, equality filter)
constexpr uint32_t SCTX_WORDS = 8, SCTX_USED = 0x80000000u, SCTX_L1 = 0xFFFFu, KIDX_NONE = 0xFFFFFFFFu;
constexpr uint64_t SBITS_MAX_BYTES = 64ull << 20;
__host__ __device__ constexpr inline uint32_t ctx_hash(uint32_t pre) {
  pre ^= pre >> 16;
  pre *= 0x7FEB352Du;
  pre ^= pre >> 15;
  return pre;
}
__host__ __device__ constexpr inline uint32_t ctx_key(uint32_t pre, uint32_t hs, uint32_t v0, uint32_t v1) {
  return ctx_hash(pre ^ ((hs + 1) * 0x27D4EB2Fu) ^ (v0 * 0x165667B1u) ^ (v1 * 0xD3A2646Cu));
}
__host__ __device__ constexpr inline uint32_t ctx_w0(uint32_t combo, uint32_t hs) { return SCTX_USED | (combo << 16) | (hs & 0xFFFFu); }
// Context filter (sbloom): a blocked Bloom filter over the contexts' keys, one 64-bit word per key
// holding 3 bits, max(16, slots / 8) words for a table of `slots` context slots (~16 bits per key).
// A request tests it before it probes the table: ~3 of 4 contexts a C3 request looks up do not
// exist, and the filter's few KB stay cached where each absent probe cost a line of the table.
__host__ __device__ constexpr inline uint32_t ctx_bloom_words(uint32_t slots) { return slots / 8 > 16 ? slots / 8 : 16; }
__host__ __device__ constexpr inline uint32_t ctx_bloom_at(uint32_t hash, uint32_t words) { return ((hash * 0x9E3779B1u) >> 7) & (words - 1); }
__host__ __device__ constexpr inline uint64_t ctx_bloom_bits(uint32_t hash) {
  uint32_t g = hash * 0x85EBCA77u;
  g ^= g >> 13;
  return (1ull << (g & 63u)) | (1ull << ((g >> 6) & 63u)) | (1ull << ((g >> 12) & 63u));
}

// 128-bit Bloom filter over entity UIDs (string-id pairs), identical on host and device.
__host__ __device__ constexpr inline uint32_t uid_bloom_bit(uint32_t et, uint32_t ei) {
  return ((et * 0x9E3779B1u) ^ (ei * 0x85EBCA77u) ^ ((ei >> 16) * 0xC2B2AE3Du)) >> 25;
}

// ---- atoms: 4-word predicates over pre-resolved (hot) attribute paths -----------------------
// A policy's when/unless clauses lower to a forward-only branch graph of atoms:
//   word0 = kind | h << 8 | t << 16 | f << 24   (t / f: next atom when true / false, or AT_SAT /
//   AT_UNSAT); word1..3 = operands. `!` swaps t and f; `&&`, `||`, boolean if-then-else and
//   clause sequencing (when: true -> next clause, false -> unsatisfied; unless: the reverse) are
//   edges. Evaluation starts at atom 0; an atom error is the policy's error. Policies without
//   conditions have no atoms and are satisfied by their scope.
enum AtomKind : uint32_t {
  AK_HAS = 1,     // hot path h present (false if only its final step is missing; error otherwise)
  AK_BOOL,        // hot h (must be bool)
  AK_EQ,          // hot h == const (w1 = tag word, w2 = y, w3 = z, register form; primitives only)
  AK_EQH,         // hot h == hot w1
  AK_INSET,       // [const primitives @record+w1 (3 words each), n = w2].contains(hot h)
  AK_CONTAINS,    // hot h (must be set).contains(const primitive w1, w2, w3)
  AK_LIKE,        // hot h (must be string) like pattern @record+w1
  AK_IS,          // var h is type w1
  AK_IN,          // var h in entity (w1 type, w2 id), w3 = bloom bit
  AK_LCMP,        // hot h (must be long) <op w1> const long (w2 lo, w3 hi); op: 0 <, 1 <=, 2 >, 3 >=
  AK_RECSET,      // hot h (must be set).containsAny([record templates]) (w3 = 0) / .contains(template) (w3 = 1);
                  // templates @record+w1 (layout: RecsetLayout), w2 = number of templates
  AK_TRUE,        // constant true (`true`; `false` is AK_TRUE with t and f swapped)
  AK_INANY,       // var h in [entity literals]: (type, id) pairs @record+w1, n = w2
  AK_EQV,         // var h == entity literal (w1 type, w2 id)
  // Inline forms (no record data: the atom's words are all it reads, plus the request's row):
  AK_LIKEI,       // hot h (must be string) like a pattern of at most one star whose literals fit 8 bytes:
                  // w1, w2 = prefix bytes then suffix bytes (little-endian), w3 = prefix length | suffix
                  // length << 4 | star << 8. Reads the string's length and its first and last 8 bytes
                  // from the row's like words (LIKE_WORDS per slot of the image's lslot_mask), staged
                  // with the hot values; from the string itself where they are not staged
  AK_INSTR,       // [string constants].contains(hot h): 1 to 3 string ids in w1..w3 (repeats fill)
};
// like words of a like slot in the request row (after the list offsets): string length, its first 8
// bytes (zero-padded), its last 8 bytes (the last byte highest; zero-padded below a short string),
// and a pad word; staged as 3 uint2 hot entries behind the hot values
constexpr uint32_t LIKE_WORDS = 6, LIKEI_MAX = 8;
constexpr uint32_t AT_UNSAT = 0xFE, AT_SAT = 0xFF, MAX_ATOMS = 0xFD;
// AK_RECSET data, all offsets relative to the policy record:
//   [n_holes, hole hot index ...]                     holes in source (evaluation) order
//   then per template: [n_keys, (key sid, field kind, a, b, c) x n_keys]   keys ascending by sid
//   field kind RF_CONST: a,b,c = register-form primitive; RF_HOLE: a = hot index;
//   RF_SETLIT: a = offset of the element list, b = element count; element = (kind, x, y, z),
//   kind RF_CONST (x,y,z register form) or RF_HOLE (x = hot index)
enum RecsetField : uint32_t { RF_CONST = 0, RF_HOLE = 1, RF_SETLIT = 2 };
constexpr uint32_t RS_FIELD_WORDS = 5, RS_ELEM_WORDS = 4;
constexpr uint32_t ATOM_WORDS = 4;

// ---- hot attribute paths ----------------------------------------------------------------------
// hot[h * HOT_WORDS] = (var, depth, key sid x MAX_PATH): var.k0.k1... (var 0 principal, 1 action,
// 2 resource, 3 context). The encoder resolves every hot path per request on the host into the
// request row: the value (memory form, refs relative to the request's heap block), or a status
// word w0 = (T_NONE tag) | HS_FINAL? | code with w1 = block offset of the error detail
// [code | aux << 8, k, et, ei] that attribute access would raise. HS_FINAL marks a failure at the
// path's last step that `has` reports as false (entity absent / attribute absent).
constexpr uint32_t HOT_WORDS = 6, MAX_PATH = 4;
constexpr uint32_t HS_FINAL = 0x100;
// ---- request rows ----------------------------------------------------------------------------
enum RowW : uint32_t {
  RW_P = 0,      // principal (type sid, id sid)
  RW_A = 2,      // action
  RW_R = 4,      // resource
  RW_PANC = 6,   // block-relative offset (signed) of the principal's ancestor (type, id) pairs
  RW_RANC = 7,
  RW_AANC = 8,
  RW_PN = 9,     // ancestor counts (AN_COUNT); an indexed image's lists hold the ancestors that are
  RW_RN = 10,    //   scope-index key entities first (AN_KEYS of them, AN_SELF: the UID itself is
  RW_AN = 11,    //   one), so the probe kernel enumerates only keys that can exist
  RW_BLK = 12,   // heap word offset of the request block
  RW_AM0 = 13,   // action mask over the image action table (`in`: the action or an ancestor), low
  RW_AM1 = 14,   //   ... high word (valid when the image's amask_ok)
  RW_ASELF = 15, // index of the action itself in the action table (`==`) in the low 16 bits (0xFFFF
                 // when absent) | the presence mask << ASELF_PRES_SHIFT (ASELF_PRES_SLOTS bits)
                 // | ASELF_CTXR: the block's RH_SCTX words hold its scope contexts
  RW_HDR = 16,   // hot slots follow: (w0, w1) per hot path
};
constexpr uint32_t MISSING_W0 = 0xFFFFFFFFu;  // level-2 index key of an absent hot value
// Set-membership level-2 keys: a policy whose satisfying evaluations all pass `hot(h).contains(c)`
// (c a primitive, or a record template of primitive constants) is filed under (h | BT_CKEY,
// element hash of c, 1), and also under (h | BT_CKEY, NOTSET_W0, 0) (a value that is no set makes
// contains raise) and, unguarded, (h | BT_CKEY, MISSING_W0, 0). A level-1 entry's word 7 (cmask)
// lists such slots. The request row then carries, after the hot slots, one word per list slot
// (the image's cslot_mask and pslot_mask: every slot a contains / containsAny atom reads, and the
// prefix-keyed ones), in slot order: the block offset of [n | CL_*, element hash x n]; slot h's
// word is at its rank among the list slots. The probe kernel probes each element of the
// request's set; contains atoms compare element hashes first and the values only on a match
// (image.h chash_*: equal values hash alike on both sides; a collision costs one exact compare).
constexpr uint32_t BT_CKEY = 0x40, NOTSET_W0 = 0xFFFFFFFEu;
constexpr uint32_t CL_MISSING = 0x80000000u, CL_NOTSET = 0x80000001u;
__host__ __device__ constexpr inline uint32_t chash_mix(uint32_t h, uint32_t x) {
  h ^= x;
  h *= 0x01000193u;
  h ^= h >> 15;
  h *= 0x2C1B3C6Du;
  return h;
}
// canonical primitive (tag, a, b): bool (T_BOOL, v, 0), long (T_LONG, lo, hi), string (T_STR,
// sid, 0), entity (T_ENT, type sid, id sid); any other value hashes its tag alone
__host__ __device__ constexpr inline uint32_t chash_prim(uint32_t tag, uint32_t a, uint32_t b) {
  return chash_mix(chash_mix(chash_mix(0x811C9DC5u, tag), a), b);
}
constexpr uint32_t CHASH_REC = 0x9747B28Cu;  // record: mix(CHASH_REC, n), then (key sid, value hash) by key
// element hash of a register-form primitive (tag word, y, z); false for other values
__host__ __device__ constexpr inline bool reg_chash(uint32_t a, uint32_t b, uint32_t c, uint32_t& out) {
  const uint32_t tag = a >> TAG_SHIFT;
  if (tag == T_BOOL || tag == T_STR) { out = chash_prim(tag, b, 0); return true; }
  if (tag == T_LONG) { out = chash_prim(T_LONG, b, c); return true; }
  if (tag == T_ENT) { out = chash_prim(T_ENT, a & X_MASK, b); return true; }
  return false;
}
// Prefix level-2 keys: a policy whose satisfying evaluations all pass `hot(h) like "lit*..."`
// (a pattern that opens with a literal) is filed in the same BT_CKEY namespace under
// (h | BT_CKEY, pfx_hash(first L literal bytes), 1), L = min(literal length, PFX_MAX); also under
// NOTSET_W0 (a value that is no string makes `like` raise) and, unguarded, MISSING_W0. The image
// keeps per slot up to PFX_LENS such lengths (Image::pfx, 0 = unused; pslot_mask lists the slots).
// For a slot of pslot_mask the request block's list holds, instead of element hashes, the value's
// prefix hashes at each of the slot's lengths it is long enough for. A slot read by any contains
// atom (cslot_mask) is never prefix-keyed, so one list per slot serves both kinds. Host-side only:
// the device probes the list's words as it probes element hashes.
constexpr uint32_t PFX_LENS = 4, PFX_MAX = 16;
constexpr uint32_t CHASH_PFX = 0x3C6EF372u;
inline uint32_t pfx_hash(const uint8_t* s, uint32_t len) {
  uint32_t h = chash_mix(CHASH_PFX, len);
  for (uint32_t k = 0; k < len; k++) h = chash_mix(h, s[k]);
  return h;
}
// RW_PN / RW_RN / RW_AN fields
constexpr uint32_t AN_COUNT = 0xFFFFu, AN_KEYS_SHIFT = 16, AN_KEYS = 0x7FFFu, AN_SELF = 0x80000000u;
constexpr uint32_t ASELF_MASK = 0xFFFFu, ASELF_CTXR = 0x80000000u;
// RW_ASELF bits 16..30: the request's presence mask over hot slots 0..14 (image.h "presence
// masks": slot h's bit when its value is present, i.e. `has` finds it); masks name no other slot
constexpr uint32_t ASELF_PRES_SHIFT = 16, ASELF_PRES_SLOTS = 15;

// ---- bytecode -------------------------------------------------------------------------------
// word0 = op | d << 8 | a << 14 | b << 20 | c << 26 (6-bit slot fields); word1 = imm
constexpr uint32_t NSLOT = 8;
constexpr uint32_t LANE_WORDS = 192;   // per-lane scratch for runtime-built sets/records
constexpr uint32_t VAL_DEPTH = 8;      // max nesting for deep equality on device
enum Op : uint32_t {
  OP_NOP = 0,
  OP_LDV,       // d = var[imm]  (0 principal, 1 action, 2 resource, 3 context)
  OP_LDC,       // d = value at cpool[imm] (2 words)
  OP_LDB,       // d = bool imm
  OP_LDS,       // d = string id imm
  OP_ATTR,      // d = a.key(imm)
  OP_HAS,       // d = a has key(imm)
  OP_EQ,        // d = a == b
  OP_NE,
  OP_LT, OP_LE, OP_GT, OP_GE,
  OP_ADD, OP_SUB, OP_MUL,
  OP_NEG,       // d = -a
  OP_NOT,       // d = !a (type-checked)
  OP_CHKB,      // error unless a is bool
  OP_JF,        // if a is false -> jump imm (a must be bool)
  OP_JT,        // if a is true  -> jump imm
  OP_JNF,       // if-then-else: if a is false jump imm (a must be bool); true falls through
  OP_JMP,       // jump imm
  OP_IN,        // d = a in b
  OP_IS,        // d = a is type(imm)
  OP_LIKE,      // d = a like pattern(cpool imm)
  OP_CONTAINS,  // d = a.contains(b)
  OP_CALL,      // d = a.containsAll(b) / containsAny(b) / isEmpty / ext methods; sub-op in c
  OP_SETNEW,    // d = new lane set with capacity imm
  OP_SETPUT,    // set d [index c] = a
  OP_RECNEW,    // d = new lane record with n=imm (keys from cpool list in next SETPUT-like ops)
  OP_RECPUT,    // rec d field c := (key imm, value a)
  OP_COND,      // end of a when/unless clause: a must be bool; c = 1 for `unless`
  OP_ERR,       // raise error: c = code, imm = aux (compile-time detected runtime error)
  OP_HOT,       // d = hot attribute slot c (pre-resolved var.attr), errors like OP_ATTR
  OP_HOTHAS,    // d = hot attribute slot c present
  OP_COUNT
};
constexpr uint32_t CHUNK_WORDS = 4096;  // policy-stream chunk staged in LDS (16 KiB)
constexpr uint32_t NHOT = 32;  // hot attribute paths per image (request-row columns; LDS per wave)
constexpr uint32_t MAX_ACT = 64;  // image action table size for per-request action masks
// OP_CALL sub-ops
enum CallOp : uint32_t {
  CO_CONTAINS_ALL = 0, CO_CONTAINS_ANY, CO_IS_EMPTY,
  CO_DEC_LT, CO_DEC_LE, CO_DEC_GT, CO_DEC_GE,
  CO_IP_V4, CO_IP_V6, CO_IP_LOOPBACK, CO_IP_MULTICAST, CO_IP_IN_RANGE,
  CO_PARSE_IP, CO_PARSE_DEC,  // ip(a) / decimal(a) over a runtime string: value into lane scratch at imm
};
// Register slots: 0..NSLOT-1 live in registers; deeper expressions spill slots NSLOT.. into the
// policy's lane scratch, 3 words each, at the end of its lane area (PW_LANE - 3 * (PW_SLOTS - NSLOT)).
constexpr uint32_t MAX_SLOTS = 64;  // 6-bit slot fields
// SETPUT / RECPUT element position: c | b << 6 (12 bits)
constexpr uint32_t MAX_LITERAL = 4096;
// Lane scratch: a private array of LANE_WORDS per lane; an image with a policy that needs more
// (big runtime literals, spilled slots) runs the stream kernel on a per-request global lane area of
// the image's lane_need words (DevBatch::lane).
constexpr uint32_t LANE_MAX = 1u << 20;
// chunk table: words field with CHUNK_GLOBAL set = one policy record too large for the LDS chunk,
// read from the policy stream in place
constexpr uint32_t CHUNK_GLOBAL = 0x80000000u;

__host__ __device__ constexpr inline uint32_t mk_ins(uint32_t op, uint32_t d, uint32_t a, uint32_t b, uint32_t c) {
  return op | (d << 8) | (a << 14) | (b << 20) | (c << 26);
}

// ---- results --------------------------------------------------------------------------------
enum Decision : uint32_t { DEC_DENY = 0, DEC_ALLOW = 1 };
// res[2r]   = decision | tier << 8 | flags << 16
// res[2r+1] = n_reasons | n_errors << 16
// RF_GENERAL: the probe kernel could not decide the request (a structural set/record
// comparison, or hits beyond even the large re-run stage); the host re-runs it on the stream
// kernel. RF_BIG: more hits than the probe kernel stages per request; re-run on its large variant.
enum ResFlags : uint32_t { RF_FORBID = 1, RF_OVERFLOW = 2, RF_VALID = 4, RF_GENERAL = 8, RF_BIG = 16 };
// A reason word with RS_CLASS set names a whole duplicate class by its representative (the first
// pass records a class hit in one slot; the host lists the members, Image::cls_off / cls_mem), so a
// request whose hits are one 150-member class fits the first pass. n_reasons counts words.
constexpr uint32_t RS_CLASS = 0x80000000u;
// error record: policy, code | aux << 8, k (string id), et (string id), ei (string id), pad
constexpr uint32_t ERR_WORDS = 6;
enum ErrCode : uint32_t {
  E_NONE = 0,
  E_TYPE = 1,            // aux = expected | got << 8 (TypeName codes below)
  E_ENTITY_MISSING = 2,  // et/ei = entity
  E_ATTR_ENTITY = 3,     // k = attribute, et/ei = entity
  E_ATTR_RECORD = 4,     // k = attribute
  E_OVERFLOW = 5,
  E_EXT = 6,             // aux = message index in image (compile-time message)
  E_DEPTH = 7,           // value nesting beyond VAL_DEPTH (device limit)
  E_LANE = 8,            // lane scratch exhausted (device limit)
  E_EXT_ARG = 9,         // aux = 0 ip / 1 decimal: the argument is not a string
  E_EXT_PARSE = 10,      // aux = 0 ip / 1 decimal, k = the string that does not parse
};
enum TypeName : uint32_t {
  TN_BOOL = 0, TN_LONG, TN_STRING, TN_ENTITY, TN_SET, TN_RECORD, TN_DECIMAL, TN_IP,
  TN_ENTITY_OR_RECORD, TN_SET_OR_ENTITY, TN_UNKNOWN,
};

// ---- image blob header (host serialization) ----------------------------------------------
constexpr uint32_t IMG_MAGIC = 0x47444543u;  // "CEDG"
constexpr uint32_t IMG_VERSION = 17;
// The blob's device region: the arrays the kernels read, each at a 256-byte-aligned blob offset
// in one contiguous range [dev_begin, dev_end) listed by a section table after the header. A device
// copy of the image is that range in one allocation (one H2D copy, one peer copy, or the blob
// itself when a collective delivered it to device memory), with each array at its blob offset.
enum DevSection : uint32_t {
  DS_PSTREAM, DS_TIER_CEND, DS_CHUNKS, DS_CPOOL, DS_GSTR_OFF, DS_HOT, DS_ACT, DS_BTAB, DS_BFILT, DS_BSTREAM,
  DS_SROWS, DS_SHASH, DS_SCTX, DS_SBITS, DS_SVALS, DS_SBLOOM, DS_GSTR_BYTES, DS_COUNT
};
constexpr uint32_t DS_ALIGN = 256;

}  // namespace cgi
