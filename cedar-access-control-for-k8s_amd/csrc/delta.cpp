// Delta images: diff, plan and host patch (delta.h). The device half is dev_blob_patch
// (cedar_eval.hip); loading and broadcasting are cg_image_load_delta (capi.cpp) and
// cg_broadcast_delta (comm.hip).
#include "delta.h"

#include <algorithm>
#include <atomic>
#include <cstring>
#include <thread>

#include "cedar.h"
#include "device.h"
#include "image.h"

namespace cg {
namespace {

// up to 16 workers over [0, n) in `grain`-sized pieces
template <class F>
void parallel_for(size_t n, size_t grain, F&& fn) {
  const size_t pieces = (n + grain - 1) / grain;
  const unsigned hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  const unsigned nt = (unsigned)std::min<size_t>(hw, pieces);
  if (nt <= 1) {
    for (size_t k = 0; k < pieces; k++) fn(k);
    return;
  }
  std::atomic<size_t> next{0};
  auto work = [&] {
    for (size_t k; (k = next.fetch_add(1)) < pieces;) fn(k);
  };
  std::vector<std::thread> ts;
  for (unsigned t = 1; t < nt; t++) ts.emplace_back(work);
  work();
  for (auto& t : ts) t.join();
}

// ---- regions: the image blob's header, device sections and host part (image.h DevSection) ----
struct Region {
  size_t nb, ne, bb, be;  // [nb, ne) of the new blob against [bb, be) of the base
  int64_t shift0 = 0;     // base offset (from bb) the comparison of nb starts at
};

// section offsets of an image blob, or false when it is not one
bool layout(const uint8_t* p, size_t n, std::vector<size_t>& cuts) {
  using namespace cgi;
  const size_t table = 16, need = table + 16 * ((size_t)DS_COUNT + 1);
  if (n < need) return false;
  uint32_t magic, version;
  std::memcpy(&magic, p, 4);
  std::memcpy(&version, p + 4, 4);
  if (magic != IMG_MAGIC || version != IMG_VERSION) return false;
  cuts.clear();
  cuts.push_back(0);
  for (uint32_t k = 0; k < DS_COUNT; k++) {
    uint64_t off;
    std::memcpy(&off, p + table + 16 * k, 8);
    if (off < cuts.back() || off > n) return false;
    cuts.push_back((size_t)off);
  }
  uint64_t end;
  std::memcpy(&end, p + table + 16 * DS_COUNT + 8, 8);
  if (end < cuts.back() || end > n) return false;
  cuts.push_back((size_t)end);
  cuts.push_back(n);
  return true;
}

// ---- the diff of one region ----
constexpr size_t BLK = 64;        // equal-run check granularity at the current shift
constexpr size_t WIN = 32;        // resync window (a shifted equal run of >= 2 * WIN bytes is found;
                                  // half a scope-index entry, whose other half may differ)
constexpr uint32_t MISS_RUN = 8;  // mismatching blocks at one shift before a search for another
constexpr uint32_t FIX_MAX = 3;   // a block differing in at most this many words: copy + word fixups
constexpr size_t AHEAD = 256;     // the short resync look-ahead after a mismatching block
constexpr uint64_t RP = 0x100000001B3ull;  // rolling-hash multiplier

struct RBuf {
  std::vector<uint64_t> ops;  // (dst, len, src) triples
  std::vector<uint8_t> lit;
  std::vector<uint32_t> fix;  // (word index, value) pairs
  void copy(size_t dst, size_t len, size_t src) {
    const size_t k = ops.size();
    if (k && !(ops[k - 1] & DL_LIT) && ops[k - 3] + ops[k - 2] == dst && ops[k - 1] + ops[k - 2] == src) {
      ops[k - 2] += len;
      return;
    }
    ops.insert(ops.end(), {dst, len, src});
  }
  void literal(size_t dst, const uint8_t* p, size_t len) {
    const size_t k = ops.size();
    if (k && (ops[k - 1] & DL_LIT) && ops[k - 3] + ops[k - 2] == dst) ops[k - 2] += len;
    else ops.insert(ops.end(), {dst, len, DL_LIT | lit.size()});
    lit.insert(lit.end(), p, p + len);
  }
};

// the base region's WIN-byte windows at WIN-aligned positions: polynomial hash -> position
struct WinIndex {
  std::vector<uint64_t> keys;  // hash | 1 (0: empty)
  std::vector<uint32_t> pos;   // window start / WIN
  std::vector<uint64_t> filt;  // one bit per hash bucket (a cheap miss test for the rolling scan)
  size_t mask = 0, fmask = 0;
  static uint64_t poly(const uint8_t* p) {
    uint64_t h = 0;
    for (size_t i = 0; i < WIN; i++) h = h * RP + p[i];
    return h;
  }
  static size_t slot(uint64_t h) { return (size_t)((h * 0x9E3779B97F4A7C15ull) >> 17); }
  void build(const uint8_t* b, size_t bl) {
    const size_t n = bl >= WIN ? (bl - WIN) / WIN + 1 : 0;
    size_t cap = 16;
    while (cap < 2 * n) cap <<= 1;
    keys.assign(cap, 0);
    pos.assign(cap, 0);
    mask = cap - 1;
    size_t fb = 1024;
    while (fb < 16 * n) fb <<= 1;
    filt.assign(fb / 64, 0);
    fmask = fb - 1;
    for (size_t j = 0; j < n; j++) {
      const uint64_t h = poly(b + j * WIN), key = h | 1;
      filt[(slot(h) & fmask) >> 6] |= 1ull << (slot(h) & 63);
      for (size_t s = slot(h) & mask;; s = (s + 1) & mask) {
        if (!keys[s]) { keys[s] = key; pos[s] = (uint32_t)j; break; }
        if (keys[s] == key) break;  // the first window with this hash stays
      }
    }
  }
  // base offset of a window with hash h, or -1
  int64_t find(uint64_t h) const {
    if (!((filt[(slot(h) & fmask) >> 6] >> (slot(h) & 63)) & 1)) return -1;
    const uint64_t key = h | 1;
    for (size_t s = slot(h) & mask; keys[s]; s = (s + 1) & mask)
      if (keys[s] == key) return (int64_t)pos[s] * (int64_t)WIN;
    return -1;
  }
};

void diff_region(const uint8_t* N, const uint8_t* B, const Region& r, RBuf& o) {
  const uint8_t* nn = N + r.nb;
  const uint8_t* bb = B + r.bb;
  const size_t nl = r.ne - r.nb, bl = r.be - r.bb;
  WinIndex ix;
  bool indexed = false;
  uint64_t pw = 1;  // RP^(WIN-1)
  for (size_t i = 1; i < WIN; i++) pw *= RP;
  int64_t shift = r.shift0;  // base position = new position + shift
  size_t pos = 0, lit_start = SIZE_MAX;
  uint32_t miss = 0;
  auto flush_lit = [&](size_t end) {
    if (lit_start != SIZE_MAX && end > lit_start) o.literal(r.nb + lit_start, nn + lit_start, end - lit_start);
    lit_start = SIZE_MAX;
  };
  while (pos < nl) {
    const size_t k = std::min(BLK, nl - pos);
    const int64_t bp = (int64_t)pos + shift;
    if (bp >= 0 && (size_t)bp + k <= bl) {
      if (std::memcmp(nn + pos, bb + bp, k) == 0) {
        flush_lit(pos);
        o.copy(r.nb + pos, k, r.bb + (size_t)bp);
        pos += k;
        miss = 0;
        continue;
      }
      // a few differing words at word-aligned positions: the block copied, those words fixed up
      if (k == BLK && (r.nb + pos) % 4 == 0 && (r.bb + (size_t)bp) % 4 == 0 && (r.nb + pos) / 4 < 0xFFFFFFFFull) {
        uint32_t nd = 0, at[FIX_MAX], val[FIX_MAX];
        for (size_t w = 0; w < BLK / 4 && nd <= FIX_MAX; w++) {
          uint32_t x, y;
          std::memcpy(&x, nn + pos + 4 * w, 4);
          std::memcpy(&y, bb + bp + 4 * w, 4);
          if (x != y) {
            if (nd < FIX_MAX) { at[nd] = (uint32_t)((r.nb + pos) / 4 + w); val[nd] = x; }
            nd++;
          }
        }
        if (nd <= FIX_MAX) {
          flush_lit(pos);
          o.copy(r.nb + pos, k, r.bb + (size_t)bp);
          for (uint32_t f = 0; f < nd; f++) o.fix.insert(o.fix.end(), {at[f], val[f]});
          pos += k;
          miss = 0;
          continue;
        }
      }
    }
    if (nl - pos < WIN + BLK || bl < WIN) {
      if (lit_start == SIZE_MAX) lit_start = pos;
      pos += k;
      continue;
    }
    // a mismatch at this shift (word fixups aside): look for the next window of the new region that
    // the base region holds (rolling hash, every byte position) and continue at that window's shift;
    // a short look ahead first (an inserted or removed entry), the rest of the region after a run of
    // MISS_RUN mismatching blocks
    if (!indexed) {
      ix.build(bb, bl);
      indexed = true;
    }
    if (lit_start == SIZE_MAX) lit_start = pos;
    const bool full = ++miss >= MISS_RUN;
    const size_t qend = full ? nl - WIN : std::min(nl - WIN, pos + AHEAD);
    size_t q = pos;
    uint64_t h = WinIndex::poly(nn + q);
    int64_t hit = -1;
    for (;;) {
      const int64_t j = ix.find(h);
      if (j >= 0 && std::memcmp(nn + q, bb + j, WIN) == 0) { hit = j; break; }
      if (q >= qend) break;
      h = (h - nn[q] * pw) * RP + nn[q + WIN];
      q++;
    }
    if (hit < 0) {
      if (full) {  // nothing of the rest is in the base region
        pos = nl;
        break;
      }
      pos += k;  // this block is literal; the next one is tried at the same shift
      continue;
    }
    // the window found is copied at once (progress even when the block around it mismatches)
    flush_lit(q);
    o.copy(r.nb + q, WIN, r.bb + (size_t)hit);
    shift = hit - (int64_t)q;
    pos = q + WIN;
    miss = 0;
  }
  flush_lit(nl);
}

}  // namespace

uint64_t blob_sum(const uint8_t* p, size_t n) {
  constexpr size_t C = 4u << 20;  // bytes per task (a multiple of 8)
  const size_t nc = (n + C - 1) / C;
  std::vector<uint64_t> part(nc, 0);
  parallel_for(nc, 1, [&](size_t k) {
    const size_t lo = k * C, hi = std::min(n, lo + C);
    uint64_t acc = 0;
    for (size_t o = lo; o < hi; o += 8) {
      uint64_t w = 0;
      std::memcpy(&w, p + o, std::min<size_t>(8, hi - o));
      acc += blob_word_mix(w, o / 8);
    }
    part[k] = acc;
  });
  uint64_t h = n;
  for (uint64_t x : part) h += x;
  return h;
}

std::vector<uint8_t> image_delta(const uint8_t* base, size_t base_len, const uint8_t* next, size_t next_len) {
  std::vector<Region> rs;
  std::vector<size_t> cn, cb;
  std::vector<Region> whole;
  if (layout(next, next_len, cn) && layout(base, base_len, cb) && cn.size() == cb.size()) {
    for (size_t k = 0; k + 1 < cn.size(); k++)
      if (cn[k + 1] > cn[k]) whole.push_back({cn[k], cn[k + 1], cb[k], cb[k + 1]});
  } else if (next_len) {
    whole.push_back({0, next_len, 0, base_len});
  }
  // regions over PIECE bytes are diffed in pieces on separate threads (C5's 49 MB head stream was
  // one thread's 20 ms): piece j of the new region against the base region's same span, widened
  // by MARGIN on both sides so that a shift across the cut still finds its match
  constexpr size_t PIECE = 4u << 20, MARGIN = 256u << 10;
  for (const Region& w : whole) {
    const size_t nl = w.ne - w.nb, bl = w.be - w.bb;
    if (nl <= PIECE) { rs.push_back(w); continue; }
    for (size_t o = 0; o < nl; o += PIECE) {
      const size_t lo = o > MARGIN ? o - MARGIN : 0, hi = std::min(bl, o + PIECE + MARGIN);
      Region r{w.nb + o, w.nb + std::min(nl, o + PIECE), w.bb + std::min(lo, bl), w.bb + std::max(std::min(lo, bl), hi)};
      r.shift0 = (int64_t)o - (int64_t)std::min(lo, bl);
      rs.push_back(r);
    }
  }
  std::vector<RBuf> out(rs.size());
  uint64_t sum = 0;
  std::thread ts([&] { sum = blob_sum(next, next_len); });
  parallel_for(rs.size(), 1, [&](size_t k) { diff_region(next, base, rs[k], out[k]); });
  ts.join();
  size_t n_ops = 0, lit = 0, n_fix = 0;
  for (auto& o : out) { n_ops += o.ops.size() / 3; lit += o.lit.size(); n_fix += o.fix.size() / 2; }
  std::vector<uint8_t> d(DL_HEAD + 24 * n_ops + 8 * n_fix + lit);
  uint8_t* w = d.data();
  auto put32 = [&](uint32_t v) { std::memcpy(w, &v, 4); w += 4; };
  auto put64 = [&](uint64_t v) { std::memcpy(w, &v, 8); w += 8; };
  put32(DL_MAGIC); put32(DL_VERSION);
  put64(base_len); put64(next_len); put64(sum); put64(n_ops); put64(lit); put64(n_fix);
  size_t lbase = 0;
  for (auto& o : out) {
    for (size_t k = 0; k < o.ops.size(); k += 3) {
      put64(o.ops[k]);
      put64(o.ops[k + 1]);
      put64((o.ops[k + 2] & DL_LIT) ? (DL_LIT | ((o.ops[k + 2] & ~DL_LIT) + lbase)) : o.ops[k + 2]);
    }
    lbase += o.lit.size();
  }
  for (auto& o : out)
    for (uint32_t v : o.fix) put32(v);
  for (auto& o : out) {
    if (!o.lit.empty()) std::memcpy(w, o.lit.data(), o.lit.size());
    w += o.lit.size();
  }
  return d;
}

DeltaPlan delta_plan(const uint8_t* d, size_t len) {
  if (!d || len < DL_HEAD) throw CedarError("truncated delta image");
  auto get32 = [&](size_t at) { uint32_t v; std::memcpy(&v, d + at, 4); return v; };
  auto get64 = [&](size_t at) { uint64_t v; std::memcpy(&v, d + at, 8); return v; };
  if (get32(0) != DL_MAGIC) throw CedarError("bad delta image magic");
  if (get32(4) != DL_VERSION) throw CedarError("unsupported delta image version");
  DeltaPlan p;
  p.base_len = get64(8);
  p.new_len = get64(16);
  p.new_sum = get64(24);
  p.n_ops = get64(32);
  const uint64_t lit = get64(40), nf = get64(48);
  if (p.n_ops > (len - DL_HEAD) / 24 || nf > (len - DL_HEAD - 24 * p.n_ops) / 8 || lit != len - DL_HEAD - 24 * p.n_ops - 8 * nf)
    throw CedarError("corrupt delta image (sizes)");
  p.fix = reinterpret_cast<const uint32_t*>(d + DL_HEAD + 24 * p.n_ops);  // (a malloc'd / bytes buffer: 8-aligned)
  p.n_fix = (size_t)nf;
  for (size_t k = 0; k < p.n_fix; k++)
    if ((uint64_t)p.fix[2 * k] * 4 + 4 > p.new_len) throw CedarError("corrupt delta image (word fixup)");
  p.lit = d + DL_HEAD + 24 * p.n_ops + 8 * nf;
  p.lit_len = (size_t)lit;
  uint64_t at = 0;
  p.pieces.reserve(3 * (p.n_ops + p.new_len / DL_PIECE + 1));
  for (uint64_t k = 0; k < p.n_ops; k++) {
    const uint64_t dst = get64(DL_HEAD + 24 * k), n = get64(DL_HEAD + 24 * k + 8), src = get64(DL_HEAD + 24 * k + 16);
    const bool is_lit = (src & DL_LIT) != 0;
    const uint64_t s = src & ~DL_LIT, lim = is_lit ? lit : p.base_len;
    if (dst != at || n == 0 || n > p.new_len - at || s > lim || n > lim - s) throw CedarError("corrupt delta image (operation)");
    for (uint64_t o = 0; o < n; o += DL_PIECE) {
      const uint64_t m = std::min<uint64_t>(DL_PIECE, n - o);
      p.pieces.insert(p.pieces.end(), {dst + o, m, src + o});
    }
    at += n;
  }
  if (at != p.new_len) throw CedarError("corrupt delta image (coverage)");
  return p;
}

std::vector<uint8_t> image_patch(const uint8_t* base, size_t base_len, const uint8_t* delta, size_t len) {
  const DeltaPlan p = delta_plan(delta, len);
  if (p.base_len != base_len) throw CedarError("delta image is for another base (length)");
  std::vector<uint8_t> out(p.new_len);
  const size_t np = p.pieces.size() / 3;
  parallel_for(np, 256, [&](size_t c) {
    for (size_t k = c * 256; k < std::min(np, c * 256 + 256); k++) {
      const uint64_t dst = p.pieces[3 * k], n = p.pieces[3 * k + 1], src = p.pieces[3 * k + 2];
      std::memcpy(out.data() + dst, (src & DL_LIT) ? p.lit + (src & ~DL_LIT) : base + src, n);
    }
  });
  for (size_t k = 0; k < p.n_fix; k++) std::memcpy(out.data() + 4 * (size_t)p.fix[2 * k], &p.fix[2 * k + 1], 4);
  if (blob_sum(out.data(), out.size()) != p.new_sum) throw CedarError("delta image does not reproduce the new image (checksum)");
  return out;
}

}  // namespace cg
