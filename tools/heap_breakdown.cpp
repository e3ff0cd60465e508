// Where a request's uploaded bytes go (no GPU): encodes SubjectAccessReview bodies against a
// compiled image (with static entities) on the direct SAR path and splits each request block into
// its header, entity table and the data behind it (attribute records, hot-slot error details,
// element-hash lists), plus the row and the ancestor-list records the batch interns.
// Build: make -C tools heap_breakdown
// Usage: heap_breakdown <policies.cedar> <static entities.json> <sars.jsonl>
#include <chrono>
#include <cstdio>
#include <fstream>
#include <sstream>

#include "../cedar-access-control-for-k8s_amd/csrc/engine.h"

using namespace cg;

static std::string slurp(const char* p) {
  std::ifstream f(p, std::ios::binary);
  std::stringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

int main(int argc, char** argv) {
  if (argc < 4) { std::fprintf(stderr, "usage: %s policies.cedar entities.json sars.jsonl\n", argv[0]); return 2; }
  DocSpec d;
  d.filename = "c3.cedar";
  d.text = slurp(argv[1]);
  const std::string ej = slurp(argv[2]);
  std::vector<EntityIn> statics;
  decode_json_entities(json_parse(ej.data(), ej.size()), statics);
  auto built = compile_image({{d}}, 1, nullptr, &statics);
  const std::vector<uint8_t> blob = built->serialize();
  auto img = Image::deserialize(blob.data(), blob.size());  // (as a loaded image: the host's sections)
  std::ifstream f(argv[3]);
  Batch b;
  b.img = img;
  double n = 0, hdr = 0, ents = 0, rest = 0, row = 0, strs = 0, fast = 0;
  EncodedRequest e;
  std::vector<std::string> lines;
  for (std::string line; std::getline(f, line);) lines.push_back(line);
  double enc_s = 0;
  for (const std::string& line : lines) {
    if (line.empty()) continue;
    e.clear();
    int fp = -1;
    std::string reason;
    const auto t0 = std::chrono::steady_clock::now();
    const int r = encode_sar_direct(*img, line.data(), line.size(), e, fp, reason);
    enc_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (r != 1) { fast++; continue; }
    n++;
    const uint32_t ne = e.blk[cgi::RH_NENT];
    hdr += cgi::RH_WORDS * 4.0;
    ents += ne * cgi::ENT_WORDS * 4.0;
    rest += (e.blk.size() - cgi::RH_WORDS - ne * cgi::ENT_WORDS) * 4.0;
    row += e.row.size() * 4.0;
    for (auto& s : e.strs) strs += (double)s.size() + 4.0;
    b.append(e);
  }
  const double heap = b.heap.size() * 4.0;
  std::printf("requests %.0f (fast path %.0f), encode %.2f us per request on one thread\n", n, fast, enc_s / (n + fast) * 1e6);
  std::printf("per request: block header %.1f B, entity table %.1f B, records / errors / lists %.1f B, row %.1f B, "
              "strings %.1f B\n", hdr / n, ents / n, rest / n, row / n, strs / n);
  std::printf("heap %.1f B per request, of which ancestor-list records %.1f B (list words %llu, shared %llu)\n", heap / n,
              (heap - (hdr + ents + rest)) / n, (unsigned long long)b.anc_words, (unsigned long long)b.anc_shared_words);
  return 0;
}
