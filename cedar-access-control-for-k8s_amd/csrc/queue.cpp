// Serving queue (include/cedargpu.h "serving queue"): turns concurrent, blocking per-request calls
// into device batches.
//
// The reference's webhook answers each SubjectAccessReview in its own goroutine with one
// PolicySet.IsAuthorized call (internal/server/authorizer/authorizer.go:36-86). Here every caller
// thread parses and converts its own request (SAR -> attributes -> fast path -> entities, the
// reference's RecordToCedarResource at authorizer.go:89) outside any lock, appends the columnar
// encoding to the open batch under the queue lock, and blocks. One flusher thread closes the open
// batch when it holds `max_batch` requests or its oldest request has waited `max_delay_us`, runs
// it (one H2D copy, one kernel launch, one D2H copy, overflow re-runs), and wakes its callers, who
// render their own decision and reason in parallel. While a batch is on the device the next one
// fills, so the batch size adapts to the offered load.
#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <thread>

#include "capi_internal.h"
#include "sar.h"

using namespace cg;
using Clock = std::chrono::steady_clock;

namespace {

struct QBatch {
  cg_batch* b = nullptr;
  Clock::time_point t0;  // arrival of the first request
  std::mutex mu;
  std::condition_variable cv;
  bool done = false;
  int rc = CG_OK;
  std::string err;
  ~QBatch() { cg_batch_destroy(b); }
};

}  // namespace

struct cg_queue {
  cg_ctx* ctx = nullptr;
  uint32_t max_batch = 4096;
  Clock::duration max_delay{};
  uint32_t max_ready = 4;  // closed batches waiting for the device before callers block
  std::mutex mu;
  std::condition_variable cv_flush, cv_space;
  std::shared_ptr<QBatch> open;
  std::deque<std::shared_ptr<QBatch>> ready;
  bool stop = false;
  std::thread flusher;
  std::string err;
  std::atomic<uint64_t> n_batches{0}, n_requests{0}, n_fast{0}, max_seen{0}, device_ns{0};

  void run();
};

void cg_queue::run() {
  for (;;) {
    std::shared_ptr<QBatch> qb;
    {
      std::unique_lock<std::mutex> g(mu);
      for (;;) {
        if (!ready.empty()) {
          qb = std::move(ready.front());
          ready.pop_front();
          cv_space.notify_all();
          break;
        }
        if (open && (stop || Clock::now() - open->t0 >= max_delay)) {
          qb = std::move(open);
          open.reset();
          break;
        }
        if (stop) return;
        if (open) cv_flush.wait_until(g, open->t0 + max_delay);
        else cv_flush.wait(g);
      }
    }
    const auto t = Clock::now();
    int rc = cg_batch_submit(qb->b);
    if (!rc) rc = cg_batch_wait(qb->b, -1);
    device_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now() - t).count();
    n_batches++;
    const uint64_t n = qb->b->items.size();
    for (uint64_t m = max_seen.load(); n > m && !max_seen.compare_exchange_weak(m, n);) {
    }
    {
      std::lock_guard<std::mutex> g(qb->mu);
      qb->rc = rc;
      if (rc) qb->err = qb->b->err;
      qb->done = true;
    }
    qb->cv.notify_all();
  }
}

namespace {

std::shared_ptr<LoadedImage> active_image(cg_ctx* ctx, std::string& err) {
  std::lock_guard<std::mutex> g(ctx->mu);
  if (!ctx->active) err = "no active image";
  return ctx->active;
}

// Appends one encoded request (encoded against `li`) to the open batch and returns the batch and
// the request's index in it. A batch holds requests of one image: a request encoded against a
// newer epoch closes the open batch first. Caller must not hold q->mu.
int enqueue(cg_queue* q, const std::shared_ptr<LoadedImage>& li, EncodedRequest& e, std::shared_ptr<QBatch>& out,
            uint32_t& idx, std::string& err) {
  std::unique_lock<std::mutex> g(q->mu);
  q->cv_space.wait(g, [q] { return q->stop || q->ready.size() < q->max_ready; });
  if (q->stop) { err = "queue closed"; return CG_E_STATE; }
  if (q->open && q->open->b->img != li) {
    q->ready.push_back(std::move(q->open));
    q->open.reset();
    q->cv_flush.notify_one();
  }
  if (!q->open) {
    auto qb = std::make_shared<QBatch>();
    qb->b = new (std::nothrow) cg_batch();
    if (!qb->b) { err = "out of host memory"; return CG_E_ARG; }
    qb->b->ctx = q->ctx;
    qb->b->img = li;
    qb->b->host.img = li->host;
    qb->t0 = Clock::now();
    q->open = std::move(qb);
    q->cv_flush.notify_one();  // arms the deadline
  }
  cg_batch* b = q->open->b;
  GUARD(err, {
    b->host.append(e);
    b->items.push_back({(int32_t)b->host.n() - 1, -1});
  })
  idx = (uint32_t)b->items.size() - 1;
  out = q->open;
  if (b->items.size() >= q->max_batch) {
    q->ready.push_back(std::move(q->open));
    q->open.reset();
    q->cv_flush.notify_one();
  }
  return CG_OK;
}

int await(std::shared_ptr<QBatch>& qb, std::string& err) {
  std::unique_lock<std::mutex> g(qb->mu);
  qb->cv.wait(g, [&] { return qb->done; });
  if (qb->rc) err = qb->err;
  return qb->rc;
}

int put_string(const std::string& s, char* buf, size_t cap, size_t* need) {
  if (need) *need = s.size() + 1;
  if (!buf) return CG_OK;
  if (cap < s.size() + 1) return CG_E_RANGE;
  std::memcpy(buf, s.c_str(), s.size() + 1);
  return CG_OK;
}

thread_local std::string t_err;

// Encodes on the calling thread, joins the open batch, waits, and renders the caller's result
// (authz: cg_batch_authz's Decision + reason; else cg_batch_decision + diagnostic).
int submit_encoded(cg_queue* q, const std::shared_ptr<LoadedImage>& li, EncodedRequest& e, int* out, char* buf,
                   size_t cap, size_t* need, bool authz) {
  std::shared_ptr<QBatch> qb;
  uint32_t idx = 0;
  int rc = enqueue(q, li, e, qb, idx, t_err);
  if (rc) return rc;
  q->n_requests++;
  if ((rc = await(qb, t_err))) return rc;
  if (authz) {
    rc = cg_batch_authz(qb->b, idx, out, buf, cap, need);
    if (rc && rc != CG_E_RANGE) t_err = qb->b->err;
    return rc;
  }
  if ((rc = cg_batch_decision(qb->b, idx, out, nullptr))) { t_err = qb->b->err; return rc; }
  if (!buf && !need) return CG_OK;
  return cg_batch_diagnostic(qb->b, idx, 0, buf, cap, need);
}

}  // namespace

extern "C" {

int cg_queue_create(cg_ctx* ctx, uint32_t max_batch, uint32_t max_delay_us, cg_queue** out) {
  if (!ctx || !out || max_batch == 0) return CG_E_ARG;
  *out = nullptr;
  auto* q = new (std::nothrow) cg_queue();
  if (!q) return CG_E_ARG;
  q->ctx = ctx;
  q->max_batch = max_batch;
  q->max_delay = std::chrono::microseconds(max_delay_us);
  try {
    q->flusher = std::thread([q] { q->run(); });
  } catch (...) {
    delete q;
    return CG_E_ARG;
  }
  *out = q;
  return CG_OK;
}

void cg_queue_destroy(cg_queue* q) {
  if (!q) return;
  {
    std::lock_guard<std::mutex> g(q->mu);
    q->stop = true;
  }
  q->cv_flush.notify_all();
  q->cv_space.notify_all();
  if (q->flusher.joinable()) q->flusher.join();  // drains ready and open batches first
  delete q;
}

const char* cg_queue_last_error(void) { return t_err.c_str(); }

int cg_queue_authorize_sar(cg_queue* q, const char* sar_json, size_t len, int* decision, char* reason, size_t cap,
                           size_t* need) {
  if (!q || !sar_json || !decision) return CG_E_ARG;
  auto li = active_image(q->ctx, t_err);
  if (!li) return CG_E_STATE;
  EncodedRequest e;
  {
    int fast = -1;
    std::string r;
    int d;
    GUARD(t_err, { d = encode_sar_direct(*li->host, sar_json, len, e, fast, r); })
    if (d == 2) {
      q->n_fast++;
      *decision = fast;
      return put_string(r, reason, cap, need);
    }
    if (d == 0) {  // the general path: JSON tree, Attributes, entities
      std::vector<EntityIn> ents;
      RequestIn req;
      GUARD(t_err, {
        JVal v = json_parse(sar_json, len);
        Attributes a = attributes_from_sar(v);
        fast = authorize_fast_path(a, r);
        if (fast >= 0) {
          q->n_fast++;
          *decision = fast;
          return put_string(r, reason, cap, need);
        }
        record_to_cedar(a, ents, req);
        encode_request(*li->host, ents, req, e);
      })
    }
  }
  return submit_encoded(q, li, e, decision, reason, cap, need, true);
}

int cg_queue_is_authorized_json(cg_queue* q, const char* item_json, size_t len, int* allow, char* diag, size_t cap,
                                size_t* need) {
  if (!q || !item_json || !allow) return CG_E_ARG;
  std::vector<EntityIn> ents;
  RequestIn req;
  GUARD(t_err, {
    JVal v = json_parse(item_json, len);
    decode_json_item(v, ents, req);
  })
  auto li = active_image(q->ctx, t_err);
  if (!li) return CG_E_STATE;
  EncodedRequest e;
  GUARD(t_err, { encode_request(*li->host, ents, req, e); })
  return submit_encoded(q, li, e, allow, diag, cap, need, false);
}

int cg_queue_stats(cg_queue* q, uint64_t* batches, uint64_t* requests, uint64_t* fast, uint64_t* max_batch,
                   uint64_t* device_ns) {
  if (!q) return CG_E_ARG;
  if (batches) *batches = q->n_batches.load();
  if (requests) *requests = q->n_requests.load();
  if (fast) *fast = q->n_fast.load();
  if (max_batch) *max_batch = q->max_seen.load();
  if (device_ns) *device_ns = q->device_ns.load();
  return CG_OK;
}

// Load generator (bench support): `threads` caller threads issue `total` blocking
// cg_queue_authorize_sar calls, cycling over sars[0..n). Reports wall seconds, latency
// percentiles (ns) and decision counts (deny, allow, no opinion).
int cg_queue_loadgen(cg_queue* q, const char* const* sars, const size_t* lens, uint32_t n, uint32_t threads,
                     uint64_t total, double* seconds, uint64_t* lat_p50, uint64_t* lat_p99, uint64_t* lat_max,
                     uint64_t* counts) {
  if (!q || !sars || !lens || !n || !threads) return CG_E_ARG;
  std::atomic<uint64_t> next{0};
  std::atomic<int> first_rc{0};
  std::mutex err_mu;
  std::string first_err;
  std::vector<std::vector<uint64_t>> lat(threads);
  std::vector<std::array<uint64_t, 3>> cnt(threads, {0, 0, 0});
  auto work = [&](uint32_t t) {
    std::vector<char> buf(4096);
    lat[t].reserve(total / threads + 1);
    for (uint64_t i; (i = next++) < total;) {
      const uint32_t k = (uint32_t)(i % n);
      int d = 0;
      size_t need = 0;
      const auto t1 = Clock::now();
      int rc = cg_queue_authorize_sar(q, sars[k], lens[k], &d, buf.data(), buf.size(), &need);
      if (rc == CG_E_RANGE) {
        buf.resize(need);
        rc = cg_queue_authorize_sar(q, sars[k], lens[k], &d, buf.data(), buf.size(), &need);
      }
      lat[t].push_back((uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now() - t1).count());
      if (rc) {
        int z = 0;
        if (first_rc.compare_exchange_strong(z, rc)) {
          std::lock_guard<std::mutex> g(err_mu);
          first_err = t_err;  // the worker's thread-local error, handed to the caller below
        }
        next = total;  // stop every worker
        return;
      }
      if (d >= 0 && d < 3) cnt[t][d]++;
    }
  };
  const auto t0 = Clock::now();
  std::vector<std::thread> ws;
  for (uint32_t t = 0; t < threads; t++) ws.emplace_back(work, t);
  for (auto& w : ws) w.join();
  if (seconds) *seconds = std::chrono::duration<double>(Clock::now() - t0).count();
  if (first_rc) {
    t_err = first_err;
    return first_rc;
  }
  std::vector<uint64_t> all;
  for (auto& l : lat) all.insert(all.end(), l.begin(), l.end());
  std::sort(all.begin(), all.end());
  auto pct = [&](double p) { return all.empty() ? 0 : all[std::min(all.size() - 1, (size_t)(p * (double)all.size()))]; };
  if (lat_p50) *lat_p50 = pct(0.50);
  if (lat_p99) *lat_p99 = pct(0.99);
  if (lat_max) *lat_max = all.empty() ? 0 : all.back();
  if (counts)
    for (int d = 0; d < 3; d++) {
      counts[d] = 0;
      for (auto& c : cnt) counts[d] += c[(size_t)d];
    }
  return CG_OK;
}

}  // extern "C"
