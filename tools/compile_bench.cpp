// Host compile-time breakdown: parse vs the whole image build (lowering, scope index, filter,
// record layout) for one policy document.  Build: make -C tools compile_bench
// Usage: compile_bench <policies.cedar>
#include <chrono>
#include <cstdio>
#include <fstream>
#include <sstream>

#include "../cedar-access-control-for-k8s_amd/csrc/engine.h"

using namespace cg;
using Clock = std::chrono::steady_clock;

int main(int argc, char** argv) {
  if (argc < 2) { std::fprintf(stderr, "usage: %s policies.cedar\n", argv[0]); return 2; }
  std::ifstream f(argv[1], std::ios::binary);
  std::stringstream ss;
  ss << f.rdbuf();
  DocSpec d;
  d.filename = "c.cedar";
  d.text = ss.str();
  d.id_prefix = "policy";
  auto t0 = Clock::now();
  auto ps = parse_policies(d.text, d.filename);
  auto t1 = Clock::now();
  auto img = compile_image({{d}}, 1);
  auto t2 = Clock::now();
  auto blob = img->serialize();
  auto t3 = Clock::now();
  auto back = Image::deserialize(blob.data(), blob.size());
  auto t4 = Clock::now();
  auto ms = [](Clock::time_point a, Clock::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
  // incremental: the same document split into 1000 parts, cached, then rebuilt
  std::vector<DocSpec> parts;
  {
    const size_t n = 1000, step = d.text.size() / n;
    size_t start = 0;
    for (size_t k = 0; k < n && start < d.text.size(); k++) {
      size_t end = k + 1 == n ? d.text.size() : d.text.find("\n\n", start + step);
      if (end == std::string::npos) end = d.text.size();
      DocSpec p;
      p.filename = "part" + std::to_string(k);
      p.text = d.text.substr(start, end - start);
      p.id_prefix = "p" + std::to_string(k) + ".";
      parts.push_back(std::move(p));
      start = end;
    }
  }
  ParseCache cache;
  auto u0 = Clock::now();
  compile_image({parts}, 1, &cache);
  auto u1 = Clock::now();
  compile_image({parts}, 2, &cache);
  auto u2 = Clock::now();
  std::printf("cached compiler over %zu documents: first build %.0f ms, rebuild %.0f ms (hits %llu)\n", parts.size(),
              ms(u0, u1), ms(u1, u2), (unsigned long long)cache.hits);
  std::printf("policies %zu: parse %.0f ms | compile_image (parse + lower + index) %.0f ms | serialize %.0f ms (%.1f MB) | "
              "deserialize %.0f ms\n", ps.size(), ms(t0, t1), ms(t1, t2), ms(t2, t3), blob.size() / 1e6, ms(t3, t4));
  return back ? 0 : 1;
}
