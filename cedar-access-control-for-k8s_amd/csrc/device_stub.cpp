// Host-memory stand-in for the device bridge (device.h), for the sanitizer builds only (make asan /
// make tsan): the host engine, C-ABI, batching layer and serving queue run unchanged against it
// under AddressSanitizer / ThreadSanitizer on a CPU. Never part of libcedargpu.so.
//
// "Evaluation" reads every input word the real upload would copy (so an out-of-bounds encode shows
// up) and writes structurally valid results: odd requests Allow with one reason (policy i mod n),
// even ones Deny with no reason, so the renderers and the C-ABI result accessors run as well.
// Completion is asynchronous like a stream: a result becomes visible only at dev_download_finish,
// after an optional jitter (CEDARGPU_STUB_JITTER_US) that exercises the queue's wait paths.
#include <cstdio>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <random>
#include <string>
#include <thread>

#include "../../include/cedargpu.h"
#include "delta.h"
#include "device.h"
#include "engine.h"

namespace cg {
using namespace cgi;

namespace {
thread_local std::string g_err;
std::atomic<uint64_t> g_sink{0};  // keeps the input reads alive
uint32_t jitter_us() {
  static const uint32_t j = [] {
    const char* e = std::getenv("CEDARGPU_STUB_JITTER_US");
    return e ? (uint32_t)std::atoi(e) : 0u;
  }();
  return j;
}
struct StubStream {
  std::mutex mu;
  uint64_t stall_us = 0;
};
}  // namespace

struct DevPool {
  int device = 0;
};

const char* dev_last_error() { return g_err.c_str(); }
int dev_count(int* n) { *n = 8; return 0; }  // contexts 0..7 (multi-context queue tests)
uint32_t dev_small_n() { return 0; }  // the stand-in has one evaluation path
int dev_select(int) { return 0; }
int dev_synchronize(int) { return 0; }

static void stub_image(int device, const Image& img, DevImage& d) {
  d.device = device;
  d.n_pol = img.n_pol();
  d.n_tiers = img.n_tiers();
  d.indexed = img.indexed;
  d.lane_need = img.lane_need;
  d.region = img.dev_end - img.dev_begin;
  d.bytes = d.region;
}
int dev_image_upload(int device, const Image& img, const uint8_t* blob, DevImage* out) {
  DevImage d;
  stub_image(device, img, d);
  d.base = std::malloc(std::max<size_t>(img.blob_len, 1));
  if (!d.base) { g_err = "out of memory"; return -5; }
  std::memcpy(d.base, blob, img.blob_len);  // the H2D copy of the whole blob
  d.origin = 0;
  d.blob_len = img.blob_len;
  *out = d;
  return 0;
}
int dev_image_copy(int device, const Image& img, const DevImage& src, DevImage* out) {
  DevImage d;
  stub_image(device, img, d);
  d.base = std::malloc(std::max<size_t>(src.blob_len, 1));
  if (!d.base) { g_err = "out of memory"; return -5; }
  std::memcpy(d.base, src.base, src.blob_len);
  d.origin = 0;
  d.blob_len = src.blob_len;
  *out = d;
  return 0;
}
int dev_blob_patch(int, const DevImage& base, const uint64_t* pieces, size_t n_pieces, const uint8_t* lit, size_t,
                   const uint32_t* fix, size_t n_fix, size_t new_len, void** out) {
  if (!base.blob_len || base.origin != 0) { g_err = "the base image has no device blob"; return -2; }
  uint8_t* nb = (uint8_t*)std::malloc(std::max<size_t>(new_len, 1));
  if (!nb) { g_err = "out of memory"; return -5; }
  for (size_t k = 0; k < n_pieces; k++) {
    const uint64_t dst = pieces[3 * k], len = pieces[3 * k + 1], src = pieces[3 * k + 2];
    std::memcpy(nb + dst, (src & DL_LIT) ? lit + (src & ~DL_LIT) : (const uint8_t*)base.base + src, len);
  }
  for (size_t k = 0; k < n_fix; k++) std::memcpy(nb + 4 * (size_t)fix[2 * k], &fix[2 * k + 1], 4);
  *out = nb;
  return 0;
}
void dev_free(int, void* p) { std::free(p); }
int dev_blob_sum(int, const void* p, size_t n, uint64_t* out) {
  *out = blob_sum((const uint8_t*)p, n);
  return 0;
}
// the stub's "device memory" is host malloc memory (cg_image_load_device callers of the stub pass it)
int dev_image_adopt(int device, const Image& img, void* dev_blob, DevImage* out) {
  DevImage d;
  stub_image(device, img, d);
  d.base = dev_blob;
  d.origin = 0;
  d.blob_len = img.blob_len;
  *out = d;
  return 0;
}
int dev_to_host(int, const void* src, size_t n, void* dst) {
  std::memcpy(dst, src, n);
  return 0;
}
void dev_image_free(DevImage* d) {
  std::free(d->base);
  *d = DevImage();
}

// (no pinned memory here: every batch array lives on the heap and is staged)
void* pinned_take(size_t) { return nullptr; }
bool pinned_give(void*, size_t) { return false; }
bool pinned_block(const void*, size_t) { return false; }
void pinned_stats(uint64_t* held_bytes, uint64_t* idle_blocks) {
  if (held_bytes) *held_bytes = 0;
  if (idle_blocks) *idle_blocks = 0;
}

int dev_pool_create(int device, DevPool** out) {
  *out = new DevPool();
  (*out)->device = device;
  return 0;
}
void dev_pool_destroy(DevPool* p) { delete p; }

int dev_batch_upload(int device, const Batch& b, DevBatch* out, void* stream, DevPool* pool) {
  DevBatch d;
  d.device = device;
  d.pool = pool;
  d.stream = stream;
  d.n = b.n();
  d.capr = b.capr;
  d.cape = b.cape;
  d.row_words = b.row_words;
  d.heap_words = b.heap.size();
  // every input section, read once (the upload's H2D copy)
  uint64_t h = 0;
  for (uint32_t x : b.heap) h = h * 31 + x;
  for (uint32_t x : b.req_base) h = h * 31 + x;
  for (uint32_t x : b.rows) h = h * 31 + x;
  for (uint32_t x : b.dev_str_off()) h = h * 31 + x;
  for (uint8_t x : b.dev_str_bytes()) h = h * 31 + x;
  g_sink += h;
  if (std::getenv("CEDARGPU_STUB_SECTIONS"))  // upload composition per section (layout studies)
    std::fprintf(stderr, "sections n=%u heap=%zu req_base=%zu rows=%zu bstr_off=%zu bstr_bytes=%zu gkeys=%zu anc=%llu shared=%llu\n",
                 b.n(), b.heap.size() * 4, b.req_base.size() * 4, b.rows.size() * 4, b.dev_str_off().size() * 4,
                 b.dev_str_bytes().size(), b.gkeys.size() * 4, (unsigned long long)b.anc_words,
                 (unsigned long long)b.anc_shared_words);
  const size_t n = std::max<uint32_t>(d.n, 1);
  const size_t words = n * 2 + 2 * n * d.capr + n * d.cape * ERR_WORDS + FU_KINDS + 1;
  d.out_bytes = words * 4;
  d.out_blk = std::calloc(words, 4);
  if (!d.out_blk) { g_err = "out of memory"; return -5; }
  d.stage = d.out_blk;  // results are read in place (bind below)
  uint32_t* w = (uint32_t*)d.out_blk;
  d.res = w;
  d.reasons_f = w + n * 2;
  d.reasons_p = d.reasons_f + n * d.capr;
  d.errs = d.reasons_p + n * d.capr;
  d.fu_cnt = d.errs + n * d.cape * ERR_WORDS;  // worklists off (cap 0): counts stay zero
  *out = d;
  return 0;
}

bool dev_batch_profile(const DevBatch&, float*, float*, float*) { return false; }

void dev_batch_free(DevBatch* d) {
  std::free(d->out_blk);
  *d = DevBatch();
}

int dev_eval(const DevImage& img, DevBatch& b, void*) {
  for (uint32_t i = 0; i < b.n; i++) {
    const bool allow = (i & 1) && img.n_pol > 0;
    b.res[2 * (size_t)i] = (allow ? DEC_ALLOW : DEC_DENY) | ((RF_VALID) << 16);
    b.res[2 * (size_t)i + 1] = allow ? 1u : 0u;
    if (allow) b.reasons_f[(size_t)i * b.capr] = i % img.n_pol, b.reasons_p[(size_t)i * b.capr] = i % img.n_pol;
  }
  b.pending = true;
  return 0;
}

int dev_time_eval(const DevImage& img, DevBatch& b, uint32_t iters, void* stream, float* ms_total) {
  const auto t0 = std::chrono::steady_clock::now();
  for (uint32_t k = 0; k < iters; k++) dev_eval(img, b, stream);
  *ms_total = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return 0;
}

int dev_time_split(const DevImage& img, DevBatch& b, uint32_t iters, void* stream, float* ms_phase, float* ms_total) {
  for (uint32_t p = 0; p < STEP_PHASES; p++) ms_phase[p] = 0.f;
  dev_time_eval(img, b, iters, stream, ms_total);
  ms_phase[PH_SCAN] = *ms_total;  // the stand-in evaluates in one host pass
  return 0;
}

int dev_subset_begin(const DevImage&, const DevBatch&, const uint32_t*, uint32_t n, uint32_t, uint32_t, int, void*,
                     DevSubset* job) {
  *job = DevSubset();
  if (n == 0) return 0;
  g_err = "stub device: the stub's results never overflow";
  return -4;
}
int dev_subset_end(DevSubset*, SubsetView* v, int64_t) { *v = SubsetView(); return 0; }
void dev_subset_release(DevSubset* job) { *job = DevSubset(); }
void dev_batch_retire(DevBatch* d, std::vector<DevSubset>& held) {
  dev_batch_free(d);  // the stand-in's work is synchronous: nothing of the batch's can still run
  for (auto& j : held) dev_subset_release(&j);
  held.clear();
}

static void bind(const DevBatch& b, Batch& host) {
  host.capr = b.capr;
  host.cape = b.cape;
  host.res = b.n ? b.res : nullptr;
  host.reasons_f = b.n ? b.reasons_f : nullptr;
  host.reasons_p = b.n ? b.reasons_p : nullptr;
  host.errs = b.n ? b.errs : nullptr;
  host.fu_cnt = b.n ? b.fu_cnt : nullptr;
  for (auto& f : host.fu) f = Batch::FollowUp();
}

int dev_download(DevBatch& b, Batch& host, void*) {
  b.pending = false;
  bind(b, host);
  return 0;
}

int dev_download_async(DevBatch& b, void* stream) {
  b.done = stream;  // "event": the stream the batch ran on
  return 0;
}

int64_t dev_now_ns() {
  return (int64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int dev_download_finish(DevBatch& b, Batch& host, int64_t deadline_ns) {
  uint64_t stall = 0;
  if (b.done) {
    StubStream* s = (StubStream*)b.done;
    std::lock_guard<std::mutex> g(s->mu);
    stall = s->stall_us;
    s->stall_us = 0;
  }
  if (const uint32_t j = jitter_us()) {
    thread_local std::minstd_rand r{std::random_device{}()};
    std::this_thread::sleep_for(std::chrono::microseconds(r() % (j + 1)));
  }
  if (stall) {
    const int64_t until = dev_now_ns() + (int64_t)stall * 1000;
    if (deadline_ns >= 0 && deadline_ns < until) {
      std::this_thread::sleep_for(std::chrono::nanoseconds(std::max<int64_t>(0, deadline_ns - dev_now_ns())));
      std::lock_guard<std::mutex> g(((StubStream*)b.done)->mu);
      ((StubStream*)b.done)->stall_us = (uint64_t)((until - dev_now_ns()) / 1000);
      return DEV_TIMEOUT;
    }
    std::this_thread::sleep_for(std::chrono::microseconds(stall));
  }
  b.pending = false;
  bind(b, host);
  return 0;
}

int dev_stall(int, void* stream, uint64_t us) {
  StubStream* s = (StubStream*)stream;
  std::lock_guard<std::mutex> g(s->mu);
  s->stall_us += std::min<uint64_t>(us, 2000000u);
  return 0;
}

int dev_stream_create(int, void** stream) {
  *stream = new StubStream();
  return 0;
}
void dev_stream_destroy(void* stream) { delete (StubStream*)stream; }
int dev_stream_sync(void*) { return 0; }

}  // namespace cg

// The collective entry points (comm.hip, RCCL) have no host stand-in: they report a device error.
extern "C" {
int cg_comm_unique_id(uint8_t*, size_t) { return CG_E_DEVICE; }
int cg_comm_create(int, int, int, const uint8_t*, size_t, cg_comm** out) {
  if (out) *out = nullptr;
  return CG_E_DEVICE;
}
void cg_comm_destroy(cg_comm*) {}
const char* cg_comm_last_error(cg_comm*) { return "no collectives in the sanitizer build"; }
int cg_broadcast_image(cg_ctx*, cg_comm*, int, const void*, size_t, uint64_t, int, size_t*) { return CG_E_DEVICE; }
int cg_broadcast_delta(cg_ctx*, cg_comm*, int, uint64_t, const void*, size_t, uint64_t, int, size_t*) { return CG_E_DEVICE; }
}
