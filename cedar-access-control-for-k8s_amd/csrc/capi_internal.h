// Internal state behind the C-ABI handles (include/cedargpu.h), shared by capi.cpp and queue.cpp.
#pragma once
#include <atomic>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/cedargpu.h"
#include "device.h"
#include "engine.h"

namespace cg {
struct LoadedImage {
  std::shared_ptr<Image> host;
  DevImage dev;
  uint64_t serial = 0;  // per-context load number (never reused, unlike the address or the epoch)
  ~LoadedImage() { dev_image_free(&dev); }
};

// Result-capacity sizing hint: what the last completed batch on an image needed. The next batch
// on that image sizes its first-pass reason capacity and its follow-up worklists by it. A hint
// only: results never depend on it (a short capacity falls back to the host re-run).
struct CapHint {
  uint64_t serial = 0;                   // LoadedImage::serial it describes (0: none)
  uint32_t ppm[FU_KINDS] = {0, 0, 0};   // share of the batch each follow-up worklist took (per million)
  uint32_t big_maxr = 0;                 // longest reason list a FU_BIG entry produced
  uint32_t gen_maxr = 0;                 // longest reason list a FU_GEN entry produced
  uint32_t first_maxr = 0;               // longest reason list (<= 64) the first pass counted exactly
};

#define GUARD(errstr, body)                                       \
  try {                                                           \
    body                                                          \
  } catch (const CedarError& e) {                                 \
    errstr = e.what();                                            \
    return CG_E_PARSE;                                            \
  } catch (const std::bad_alloc&) {                               \
    errstr = "out of host memory";                                \
    return CG_E_ARG;                                              \
  } catch (const std::exception& e) {                             \
    errstr = e.what();                                            \
    return CG_E_ARG;                                              \
  }

// Result readers over device output (Batch::reason_ids, diagnostic_json): a malformed result word
// (e.g. a reason naming no duplicate class) is a device fault, reported as CG_E_DEVICE, never an
// exception across the C ABI.
#define GUARD_RESULT(errstr, body)                                \
  try {                                                           \
    body                                                          \
  } catch (const std::bad_alloc&) {                               \
    errstr = "out of host memory";                                \
    return CG_E_ARG;                                              \
  } catch (const std::exception& e) {                             \
    errstr = std::string("malformed device result: ") + e.what(); \
    return CG_E_DEVICE;                                           \
  }

}  // namespace cg

using cg::LoadedImage;

struct cg_batch;
namespace cg {
// cg_batch_wait with separate deadlines (steady-clock ns, < 0 none) for the results' download and
// for the host re-runs after it: the serving queue polls the download in short slices (so that
// closing the queue over a hung device stays bounded) without giving a re-run only a slice's time.
int batch_wait(cg_batch* b, int64_t download_deadline, int64_t rerun_deadline);
}  // namespace cg

struct cg_ctx {
  int device = 0;
  void* stream = nullptr;
  // host-driven re-runs (rare) run on their own stream, so that a pipelined next batch queued on
  // `stream` does not delay them (and they do not delay it)
  void* rstream = nullptr;
  cg::DevPool* pool = nullptr;  // batch buffers (device + pinned staging), reused across batches
  std::mutex mu;
  std::map<uint64_t, std::shared_ptr<LoadedImage>> images;
  std::shared_ptr<LoadedImage> active;
  std::string err;
  uint64_t next_serial = 1;  // under mu
  cg::CapHint hint;          // under mu
  // cg_ctx_inject_fault: submits left to fail, and the device stall before each batch (us)
  std::atomic<uint64_t> fault_errors{0}, fault_stall_us{0}, fault_kidx{0};
  std::atomic<uint64_t> activations{0};  // cg_image_activate switches (cg_queue_metrics)
};

struct cg_batch {
  cg_ctx* ctx = nullptr;
  std::shared_ptr<LoadedImage> img;
  cg::Batch host;
  cg::DevBatch dev;
  bool submitted = false, done = false;
  bool downloaded = false;  // the first pass's results (and follow-ups) are in the pinned block
  int failed = 0;        // a host re-run missed its deadline: every later wait returns this
  uint32_t n_rerun = 0;  // requests re-run by cg_batch_wait
  // cg_batch_route: (slot << 8 | CG_ROUTE_* bit) per request a follow-up worklist or a host re-run
  // finished, appended by the fold (27k of C3's 1M), sorted on the first query
  std::vector<uint64_t> routes;
  bool routes_sorted = false;
  uint32_t n_fu[cg::FU_KINDS] = {0, 0, 0};  // requests finished by each on-device follow-up worklist
  std::string err;
  // items: caller-visible entries; dev >= 0 is the device request index, else a fast-path result
  struct Item { int32_t dev; int32_t fast; };
  std::vector<Item> items;
  std::map<uint32_t, std::string> fast_reason;  // authz fast paths: the reason; admission: error text
  std::vector<cg::DevSubset> held;  // re-run result blocks the host lists point into (Batch::big)
  // cg_batch_set_profile: host intervals of submit (finalize, group, upload call, launch + D2H
  // enqueue) and of the wait (ms), filled as they pass
  double prof_ms[5] = {0, 0, 0, 0, 0};
  ~cg_batch() {
    if (dev.direct && dev.pending) {
      // inputs were copied straight from these arrays (pinned blocks) and the copy may still run:
      // they go with the retired batch and return to the pinned pool once its stream drains
      // (dstr_off / dstr_bytes: the device string table of an all-atomic image, uploaded in place
      // of bstr_* and as liable to be copied straight from its pinned block)
      struct Arrays {
        cg::PinVec<uint32_t> heap, req_base, rows, gkeys, bstr_off, dstr_off;
        cg::PinVec<uint8_t> bstr_bytes, dstr_bytes;
      };
      try {
        auto a = std::make_shared<Arrays>();
        a->heap.swap(host.heap); a->req_base.swap(host.req_base); a->rows.swap(host.rows);
        a->gkeys.swap(host.gkeys); a->bstr_off.swap(host.bstr_off); a->bstr_bytes.swap(host.bstr_bytes);
        a->dstr_off.swap(host.dstr_off); a->dstr_bytes.swap(host.dstr_bytes);
        dev.keep = std::move(a);
        cg::g_pinned_kept.fetch_add(1, std::memory_order_relaxed);
      } catch (...) {
        cg::dev_batch_free(&dev);  // (drains the stream first)
      }
    }
    dev_batch_retire(&dev, held);  // never waits: blocks still in use return once the stream drains
  }
  int32_t dev_of(uint32_t i) const { return i < items.size() ? items[i].dev : -1; }
};

