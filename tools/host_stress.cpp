// Host-side stress driver for the sanitizer builds (csrc/Makefile `asan` / `tsan`): the compiler,
// JSON decoders, SAR / admission models, batch C-ABI and serving queue, linked against the
// host-memory device stand-in (csrc/device_stub.cpp), under AddressSanitizer+UBSan or
// ThreadSanitizer on the CPU. Exit status 0 = every phase ran and every call returned a defined
// status; the sanitizers abort on the first report.
//
//   phases: compile (multi-tier, static entities, bad documents, incremental rebuilds)
//           decode  (valid and mutated JSON through every batch entry point, results read back)
//           batches (concurrent batch create / submit / wait / read on one context)
//           queue   (caller threads on the serving queue while images reload and faults fire)
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../include/cedargpu.h"

static int g_fail = 0;
#define CHECK(c, ...)                                   \
  do {                                                  \
    if (!(c)) {                                         \
      std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      std::fprintf(stderr, __VA_ARGS__);                \
      std::fprintf(stderr, "\n");                       \
      g_fail++;                                         \
    }                                                   \
  } while (0)

static const char* VERBS[] = {"get", "list", "watch", "create", "update", "patch", "delete"};
static const char* RES[] = {"pods", "secrets", "configmaps", "deployments", "services", "nodes"};

static std::string abac_policies(int n, std::mt19937& r) {
  std::string out;
  for (int i = 0; i < n; i++) {
    const int g = (int)(r() % 50), ns = (int)(r() % 20);
    switch (r() % 5) {
      case 0:
        out += "permit (principal in k8s::Group::\"g" + std::to_string(g) + "\", action in [k8s::Action::\"get\", k8s::Action::\"list\"],"
               " resource is k8s::Resource) when { resource has namespace && resource.namespace == \"ns" + std::to_string(ns) + "\" };\n";
        break;
      case 1:
        out += "forbid (principal in k8s::Group::\"g" + std::to_string(g) + "\", action in [k8s::Action::\"delete\"], resource is k8s::Resource)"
               " when { resource has name && resource.name like \"prod-*\" };\n";
        break;
      case 2:
        out += "permit (principal, action, resource is k8s::Resource) when { resource.resource == \"" + std::string(RES[r() % 6]) +
               "\" && principal.name like \"user-1*\" };\n";
        break;
      case 3:  // bytecode: runtime ip(), records
        out += "permit (principal, action, resource) when { context has ip && ip(context.ip).isInRange(ip(\"10.0.0.0/8\")) };\n";
        break;
      default:
        out += "permit (principal is k8s::User, action == k8s::Action::\"get\", resource is k8s::NonResourceURL)"
               " when { resource.path like \"/healthz*\" };\n";
    }
  }
  return out;
}

static std::string sar_json(std::mt19937& r) {
  const int u = (int)(r() % 200), g = (int)(r() % 50), ns = (int)(r() % 20);
  std::string s = "{\"apiVersion\":\"authorization.k8s.io/v1\",\"kind\":\"SubjectAccessReview\",\"spec\":{\"user\":\"user-" +
                  std::to_string(u) + "\",\"uid\":\"" + std::to_string(u) + "\",\"groups\":[\"g" + std::to_string(g) + "\",\"g" +
                  std::to_string((g * 7) % 50) + "\"],";
  if (r() % 8 == 0)
    s += "\"nonResourceAttributes\":{\"path\":\"/healthz\",\"verb\":\"get\"}}}";
  else
    s += "\"resourceAttributes\":{\"verb\":\"" + std::string(VERBS[r() % 7]) + "\",\"namespace\":\"ns" + std::to_string(ns) +
         "\",\"group\":\"\",\"version\":\"v1\",\"resource\":\"" + RES[r() % 6] + "\",\"name\":\"" + (r() % 3 ? "web" : "prod-db") +
         "\"}}}";
  return s;
}

static std::string review_json(std::mt19937& r, int i) {
  const std::string kind = r() % 2 ? "ConfigMap" : "Secret";
  return "{\"apiVersion\":\"admission.k8s.io/v1\",\"kind\":\"AdmissionReview\",\"request\":{\"uid\":\"" + std::to_string(i) +
         "\",\"kind\":{\"group\":\"\",\"version\":\"v1\",\"kind\":\"" + kind + "\"},\"resource\":{\"group\":\"\",\"version\":\"v1\","
         "\"resource\":\"" + (kind == "Secret" ? "secrets" : "configmaps") + "\"},\"name\":\"n" + std::to_string(i) +
         "\",\"namespace\":\"ns1\",\"operation\":\"CREATE\",\"userInfo\":{\"username\":\"user-" + std::to_string(r() % 9) +
         "\",\"groups\":[\"g1\"]},\"object\":{\"apiVersion\":\"v1\",\"kind\":\"" + kind + "\",\"metadata\":{\"name\":\"n" +
         std::to_string(i) + "\",\"namespace\":\"ns1\",\"labels\":{\"owner\":\"user-" + std::to_string(r() % 9) +
         "\",\"a\":\"b\"}},\"data\":{\"k\":\"v\"}}}}";
}

static std::string entities_json() {
  std::string s = "[";
  for (int g = 0; g < 50; g++) {
    if (g) s += ",";
    s += "{\"uid\":{\"type\":\"k8s::Group\",\"id\":\"g" + std::to_string(g) + "\"},\"attrs\":{},\"parents\":[";
    if (g >= 5) s += "{\"type\":\"k8s::Group\",\"id\":\"g" + std::to_string(g / 5) + "\"}";
    s += "]}";
  }
  return s + "]";
}

static std::vector<uint8_t> build(cg_compiler* c, uint64_t epoch, int n_pol, std::mt19937& r, bool broken) {
  cg_compiler_clear(c);
  cg_compiler_add_tier(c);
  const std::string p = abac_policies(n_pol, r);
  CHECK(cg_compiler_add_document(c, "c3.cedar", p.data(), p.size(), "policy", "") == 0, "add doc");
  cg_compiler_add_tier(c);
  for (int t = 0; t < 20; t++) {
    std::string d = t == 7 && broken ? "permit (principal, action, resource) when { 1 + };" : abac_policies(5, r);
    const std::string name = "tenant-" + std::to_string(t);
    CHECK(cg_compiler_add_document_ex(c, name.c_str(), d.data(), d.size(), name.c_str(), "-uid", CG_DOC_SKIP_INVALID) == 0, "add crd");
  }
  const std::string ents = entities_json();
  CHECK(cg_compiler_set_entities(c, ents.data(), ents.size()) == 0, "entities");
  uint8_t* img = nullptr;
  size_t len = 0;
  const int rc = cg_compiler_build(c, epoch, &img, &len);
  CHECK(rc == 0, "build: %s", cg_compiler_last_error(c));
  std::vector<uint8_t> out(img, img + len);
  cg_free(img);
  char buf[4096];
  size_t need = 0;
  CHECK(cg_compiler_doc_errors(c, buf, sizeof buf, &need) == 0, "doc errors");
  return out;
}

static void read_batch(cg_batch* b, int kind) {
  const uint32_t n = cg_batch_size(b);
  std::vector<char> buf(1 << 16);
  for (uint32_t i = 0; i < n; i++) {
    size_t need = 0;
    if (kind == 0) {
      int allow = 0;
      uint32_t tier = 0;
      CHECK(cg_batch_decision(b, i, &allow, &tier) == 0, "decision");
      CHECK(cg_batch_diagnostic(b, i, 0, buf.data(), buf.size(), &need) == 0, "diag");
    } else if (kind == 1) {
      int dec = 0;
      CHECK(cg_batch_authz(b, i, &dec, buf.data(), buf.size(), &need) == 0, "authz");
    } else {
      int allowed = 0, code = 0;
      CHECK(cg_batch_admit(b, i, &allowed, &code, buf.data(), buf.size(), &need) == 0, "admit");
    }
  }
}

static void phase_decode(cg_ctx* ctx, std::mt19937& r) {
  for (int round = 0; round < 60; round++) {
    const int kind = round % 3;
    std::string payload = "[";
    for (int i = 0; i < 40; i++) {
      if (i) payload += ",";
      if (kind == 0) {
        payload += "{\"entities\":[{\"uid\":{\"type\":\"k8s::User\",\"id\":\"user-" + std::to_string(i) +
                   "\"},\"attrs\":{\"name\":\"user-1" + std::to_string(i) + "\"},\"parents\":[{\"type\":\"k8s::Group\",\"id\":\"g" +
                   std::to_string(i % 50) + "\"}]}],\"request\":{\"principal\":{\"type\":\"k8s::User\",\"id\":\"user-" +
                   std::to_string(i) + "\"},\"action\":{\"type\":\"k8s::Action\",\"id\":\"get\"},\"resource\":{\"type\":"
                   "\"k8s::Resource\",\"id\":\"/api/v1/pods\"},\"context\":{\"ip\":\"10.1.2." + std::to_string(i) + "\"}}}";
      } else if (kind == 1) {
        payload += sar_json(r);
      } else {
        payload += review_json(r, i);
      }
    }
    payload += "]";
    // every third round: mutate (truncate / flip bytes / splice)
    if (round % 3 == 2) {
      const int m = (int)(r() % 3);
      if (m == 0) payload.resize(r() % payload.size());
      else if (m == 1) for (int k = 0; k < 8; k++) payload[r() % payload.size()] = (char)(r() % 128);
      else payload.insert(r() % payload.size(), "{\"x\":[1,2,{\"y\":");
    }
    cg_batch* b = nullptr;
    CHECK(cg_batch_create(ctx, &b) == 0, "batch create");
    const int rc = kind == 0 ? cg_batch_add_json(b, payload.data(), payload.size())
                 : kind == 1 ? cg_batch_add_sar_json(b, payload.data(), payload.size())
                             : cg_batch_add_admission_json(b, payload.data(), payload.size());
    if (rc == 0 && cg_batch_size(b) > 0) {
      CHECK(cg_batch_submit(b) == 0, "submit: %s", cg_last_error(ctx));
      CHECK(cg_batch_wait(b, -1) == 0, "wait: %s", cg_last_error(ctx));
      read_batch(b, kind);
    }
    cg_batch_destroy(b);
  }
  // per-item conversions
  for (int i = 0; i < 200; i++) {
    std::string s = sar_json(r);
    if (i % 4 == 3) s.resize(r() % s.size());
    char out[8192];
    size_t need = 0;
    (void)cg_sar_to_cedar_json(s.data(), s.size(), out, sizeof out, &need);
    std::string a = review_json(r, i);
    if (i % 4 == 3) a[r() % a.size()] = '"';
    (void)cg_admission_to_cedar_json(a.data(), a.size(), out, sizeof out, &need);
  }
}

static void phase_batches(cg_ctx* ctx) {
  std::vector<std::thread> th;
  for (int t = 0; t < 6; t++)
    th.emplace_back([ctx, t] {
      std::mt19937 r(100 + t);
      for (int k = 0; k < 40; k++) {
        std::string payload = "[";
        const int n = 1 + (int)(r() % 300);
        for (int i = 0; i < n; i++) payload += (i ? "," : "") + sar_json(r);
        payload += "]";
        cg_batch* b = nullptr;
        CHECK(cg_batch_create(ctx, &b) == 0, "create");
        CHECK(cg_batch_add_sar_json(b, payload.data(), payload.size()) == 0, "add: %s", cg_last_error(ctx));
        if (cg_batch_size(b)) {
          CHECK(cg_batch_submit(b) == 0, "submit");
          if (k % 5 == 4) { cg_batch_destroy(b); continue; }  // destroyed while in flight
          CHECK(cg_batch_wait(b, -1) == 0, "wait");
          read_batch(b, 1);
        }
        cg_batch_destroy(b);
      }
    });
  for (auto& x : th) x.join();
}

static void phase_queue(cg_ctx* ctx, cg_compiler* comp, std::mt19937& r0) {
  cg_queue* q = nullptr;
  CHECK(cg_queue_create(ctx, 64, 50, &q) == 0, "queue");
  std::atomic<bool> stop{false};
  std::atomic<uint64_t> ok{0}, timeouts{0}, device_err{0};
  std::thread reloader([&] {
    std::mt19937 r(7);
    uint64_t epoch = 10;
    while (!stop.load()) {
      const auto img = build(comp, epoch, 50 + (int)(r() % 50), r, epoch % 2);
      CHECK(cg_image_load(ctx, img.data(), img.size(), epoch) == 0, "load");
      CHECK(cg_image_activate(ctx, epoch) == 0, "activate");
      if (epoch > 10) cg_image_unload(ctx, epoch - 1);
      epoch++;
      std::this_thread::sleep_for(std::chrono::milliseconds(3));
    }
  });
  std::thread faults([&] {
    std::mt19937 r(8);
    while (!stop.load()) {
      const int k = (int)(r() % 3);
      cg_ctx_inject_fault(ctx, k == 0 ? CG_FAULT_NONE : k == 1 ? CG_FAULT_DEVICE_ERROR : CG_FAULT_STALL, k == 1 ? 2 : 300);
      std::this_thread::sleep_for(std::chrono::milliseconds(2));
    }
    cg_ctx_inject_fault(ctx, CG_FAULT_NONE, 0);
  });
  std::vector<std::thread> callers;
  for (int t = 0; t < 24; t++)
    callers.emplace_back([&, t] {
      std::mt19937 r(1000 + t);
      char reason[8192];
      for (int k = 0; k < 400; k++) {
        const std::string s = sar_json(r);
        int dec = -1;
        size_t need = 0;
        const int64_t timeout = k % 4 == 0 ? 200000 : 50000000;  // 0.2 ms / 50 ms
        const int rc = cg_queue_authorize_sar(q, s.data(), s.size(), timeout, &dec, reason, sizeof reason, &need);
        if (rc == CG_OK) { ok++; CHECK(dec >= 0 && dec <= 2, "decision %d", dec); }
        else if (rc == CG_E_TIMEOUT) timeouts++;
        else if (rc == CG_E_DEVICE) device_err++;
        else CHECK(false, "queue rc %d: %s", rc, cg_queue_last_error());
      }
    });
  for (auto& x : callers) x.join();
  stop = true;
  reloader.join();
  faults.join();
  uint64_t batches = 0, requests = 0, fast = 0, maxb = 0, waits = 0;
  cg_queue_stats(q, &batches, &requests, &fast, &maxb, &waits);
  std::printf("queue: ok %llu timeouts %llu device errors %llu | batches %llu requests %llu max batch %llu\n",
              (unsigned long long)ok.load(), (unsigned long long)timeouts.load(), (unsigned long long)device_err.load(),
              (unsigned long long)batches, (unsigned long long)requests, (unsigned long long)maxb);
  CHECK(ok.load() > 0, "no call succeeded");
  cg_queue_destroy(q);
}

// four contexts behind one queue: images reach the others by cg_image_load_peer, later than the
// first context's activation (batches fall back to the first context meanwhile)
static void phase_multi(cg_compiler* comp) {
  std::mt19937 r(77);
  cg_ctx* ctxs[4] = {};
  for (int k = 0; k < 4; k++) CHECK(cg_ctx_create(k, &ctxs[k]) == 0, "ctx %d", k);
  auto img = build(comp, 500, 120, r, false);
  CHECK(cg_image_load(ctxs[0], img.data(), img.size(), 500) == 0, "load");
  CHECK(cg_image_activate(ctxs[0], 500) == 0, "activate");
  for (int k = 1; k < 4; k++) CHECK(cg_image_load_peer(ctxs[k], ctxs[0], 500) == 0, "peer load %d", k);
  cg_queue* q = nullptr;
  CHECK(cg_queue_create_multi(ctxs, 4, 32, 20, &q) == 0, "queue multi");
  std::atomic<bool> stop{false};
  std::thread reloader([&] {
    std::mt19937 rr(5);
    for (uint64_t epoch = 501; !stop.load(); epoch++) {
      auto im = build(comp, epoch, 60 + (int)(rr() % 60), rr, false);
      CHECK(cg_image_load(ctxs[0], im.data(), im.size(), epoch) == 0, "load");
      CHECK(cg_image_activate(ctxs[0], epoch) == 0, "activate");
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
      for (int k = 1; k < 4; k++) {
        CHECK(cg_image_load_peer(ctxs[k], ctxs[0], epoch) == 0, "peer load");
        cg_image_unload(ctxs[k], epoch - 1);
      }
      cg_image_unload(ctxs[0], epoch - 1);
      std::this_thread::sleep_for(std::chrono::milliseconds(2));
    }
  });
  std::atomic<uint64_t> ok{0};
  std::vector<std::thread> callers;
  for (int t = 0; t < 16; t++)
    callers.emplace_back([&, t] {
      std::mt19937 rt(300 + t);
      char reason[8192];
      for (int k = 0; k < 300; k++) {
        const std::string s = sar_json(rt);
        int dec = -1;
        size_t need = 0;
        const int rc = cg_queue_authorize_sar(q, s.data(), s.size(), -1, &dec, reason, sizeof reason, &need);
        CHECK(rc == CG_OK, "multi queue rc %d: %s", rc, cg_queue_last_error());
        if (rc == CG_OK) ok++;
      }
    });
  for (auto& x : callers) x.join();
  stop = true;
  reloader.join();
  uint64_t used = 0;
  for (uint32_t k = 0; k < 4; k++) {
    uint64_t b = 0, n = 0;
    cg_queue_gpu_stats(q, k, &b, &n);
    std::printf("  context %u: %llu batches, %llu requests\n", k, (unsigned long long)b, (unsigned long long)n);
    used += b > 0;
  }
  CHECK(used >= 2, "batches went to %llu contexts only", (unsigned long long)used);
  cg_queue_destroy(q);
  for (auto* c : ctxs) cg_ctx_destroy(c);
}

int main() {
  std::mt19937 r(1);
  cg_compiler* comp = nullptr;
  CHECK(cg_compiler_create(&comp) == 0, "compiler");
  for (int k = 0; k < 6; k++) build(comp, 1 + k, 200, r, k % 2);  // incremental rebuilds (parse cache)
  std::printf("compile ok\n");
  cg_ctx* ctx = nullptr;
  CHECK(cg_ctx_create(0, &ctx) == 0, "ctx");
  const auto img = build(comp, 9, 300, r, true);
  CHECK(cg_image_load(ctx, img.data(), img.size(), 9) == 0, "load: %s", cg_last_error(ctx));
  CHECK(cg_image_activate(ctx, 9) == 0, "activate");
  phase_decode(ctx, r);
  std::printf("decode ok\n");
  phase_batches(ctx);
  std::printf("batches ok\n");
  phase_queue(ctx, comp, r);
  std::printf("queue ok\n");
  phase_multi(comp);
  std::printf("multi-context queue ok\n");
  cg_ctx_destroy(ctx);
  cg_compiler_destroy(comp);
  std::printf("%s (%d failures)\n", g_fail ? "FAILED" : "PASSED", g_fail);
  return g_fail ? 1 : 0;
}
