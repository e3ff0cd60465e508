// Serving queue (include/cedargpu.h "serving queue"): turns concurrent, blocking per-request calls
// into device batches, over one GPU or several in one process.
//
// The reference's webhook answers each SubjectAccessReview in its own goroutine with one
// PolicySet.IsAuthorized call (internal/server/authorizer/authorizer.go:36-86, server.go:67-117).
// Here every caller thread parses, converts and encodes its own request (SAR -> attributes -> fast
// path -> entities -> position-independent request block) with no lock held, hands the block to one
// of 16 stripes (a mutex held for one pointer push) and sleeps. One flusher thread drains the
// stripes into device batches (at most `max_batch` requests; with `max_delay_us` > 0 it first lets
// a batch fill for that long after its first request) and deals each closed batch to the least
// loaded GPU: one submitter thread per context runs its batches (submit, wait; the next batch is
// submitted before the previous one is waited for) and publishes the results with one futex wake
// for every waiting caller. While every GPU is busy with a batch and
// has the next one queued, the flusher keeps draining into a larger batch, so the batch size adapts
// to the offered load. Callers render their own decision and reason in parallel.
//
// Requests are encoded against the first context's active image; a batch dealt to another context
// runs on that context's image of the same epoch (loaded with cg_image_load_peer, or the same blob),
// or goes to the first context while another has not loaded that epoch yet.
#include <linux/futex.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <climits>
#include <condition_variable>
#include <cstring>
#include <ctime>
#include <deque>
#include <mutex>
#include <thread>

#include "capi_internal.h"
#include "sar.h"

using namespace cg;
using Clock = std::chrono::steady_clock;

namespace {

struct Ticket;

struct QBatch {
  cg_batch* b = nullptr;
  Clock::time_point t_submit{};  // batch latency: submit -> results published
  int rc = CG_OK;
  std::string err;
  std::vector<std::shared_ptr<Ticket>> tickets;  // released (cleared) when the batch is published
  ~QBatch() { cg_batch_destroy(b); }
};

// One caller's request. Shared by the caller and the flusher / submitter: a caller whose deadline
// passes returns while the queue may still hold (and batch) its ticket.
struct Ticket {
  std::shared_ptr<LoadedImage> img;  // the image the request was encoded against (first context)
  EncodedRequest e;
  Clock::time_point t;
  // set by the flusher before the batch is dealt; read by the caller once `ready`
  std::shared_ptr<QBatch> qb;
  uint32_t idx = 0;
  std::atomic<uint32_t> ready{0};  // the request's batch is published
  // T_QUEUED until the flusher takes the ticket into a batch (T_TAKEN), or the caller gives up
  // first (T_ABANDONED: its deadline passed while it was still queued; the flusher drops it, so
  // a stalled GPU's backlog is not evaluated for callers that already failed safe)
  std::atomic<uint32_t> state{0};
  int rc = CG_OK;    // a request the batch could not take (error set, no batch)
  std::string err;
};
constexpr uint32_t T_QUEUED = 0, T_TAKEN = 1, T_ABANDONED = 2;

constexpr uint32_t STRIPES = 16;

using TicketP = std::shared_ptr<Ticket>;

struct alignas(64) Stripe {
  std::mutex mu;
  std::vector<TicketP> q;
};

// Futex on a 32-bit publication counter: callers sleep on it with an optional timeout (C++20
// atomic wait has none), the flusher wakes them all once per published batch.
void futex_wake_all(std::atomic<uint32_t>* w) {
  (void)syscall(SYS_futex, reinterpret_cast<uint32_t*>(w), FUTEX_WAKE_PRIVATE, INT_MAX, nullptr, nullptr, 0);
}
void futex_wait(std::atomic<uint32_t>* w, uint32_t seen, int64_t rel_ns) {
  timespec ts{(time_t)(rel_ns / 1000000000), (long)(rel_ns % 1000000000)};
  (void)syscall(SYS_futex, reinterpret_cast<uint32_t*>(w), FUTEX_WAIT_PRIVATE, seen, rel_ns < 0 ? nullptr : &ts, nullptr, 0);
}
int64_t now_ns() {
  return (int64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now().time_since_epoch()).count();
}

// cg_queue_metrics' latency buckets (ns, "le"): 10 us .. 10 s, holding the reference's
// request_duration_seconds buckets (metrics.go:43: 0.25, 0.5, 0.7, 1, 1.5, 3, 5, 10 s)
constexpr uint64_t k_lat_bounds[CG_LAT_BOUNDS] = {
    10000,     25000,     50000,      100000,     250000,     500000,     1000000,
    2500000,   5000000,   10000000,   25000000,   50000000,   100000000,  250000000,
    500000000, 700000000, 1000000000, 1500000000, 3000000000, 5000000000, 10000000000};
uint32_t lat_bucket(uint64_t ns) {
  return (uint32_t)(std::lower_bound(k_lat_bounds, k_lat_bounds + CG_LAT_BOUNDS, ns) - k_lat_bounds);
}
uint32_t size_bucket(uint64_t n) {
  uint32_t k = 0;
  while (k < CG_BATCH_BUCKETS && (1ull << k) < n) k++;
  return k;
}

// the serving metrics (relaxed counters; a few atomics per call)
struct QMetrics {
  std::atomic<uint64_t> req[4]{}, lat[4][CG_LAT_BOUNDS + 1]{}, lat_sum[4]{};
  std::atomic<uint64_t> bsize[CG_BATCH_BUCKETS + 1]{}, blat[CG_LAT_BOUNDS + 1]{}, blat_sum{0};
  void request(uint32_t outcome, uint64_t ns) {
    if (outcome > 3) return;
    req[outcome].fetch_add(1, std::memory_order_relaxed);
    lat[outcome][lat_bucket(ns)].fetch_add(1, std::memory_order_relaxed);
    lat_sum[outcome].fetch_add(ns, std::memory_order_relaxed);
  }
};

}  // namespace

// one GPU's submitter: runs the batches dealt to its context, in order
struct QWorker {
  cg_ctx* ctx = nullptr;
  std::thread th;
  std::mutex mu;
  std::condition_variable cv;
  std::deque<std::shared_ptr<QBatch>> q;
  std::atomic<uint32_t> load{0};  // batches queued or running
  bool stop = false;              // under mu
  std::atomic<uint64_t> n_batches{0}, n_requests{0};
};

struct cg_queue {
  std::vector<cg_ctx*> ctxs;  // ctxs[0] encodes (its active image)
  uint32_t max_batch = 4096;
  Clock::duration max_delay{};
  Stripe stripes[STRIPES];
  std::atomic<uint32_t> pending{0};     // tickets in the stripes (the flusher sleeps on it at 0)
  std::atomic<uint32_t> pub{0};         // bumped per publication (callers' futex word)
  std::atomic<uint32_t> next_stripe{0};
  std::atomic<bool> stop{false};
  std::thread flusher;
  std::vector<std::unique_ptr<QWorker>> workers;
  std::mutex slot_mu;  // the flusher waits here for a submitter with room
  std::condition_variable slot_cv;
  std::atomic<uint64_t> n_batches{0}, n_requests{0}, n_fast{0}, max_seen{0}, device_ns{0}, n_abandoned{0};
  std::atomic<int64_t> stop_ns{0};  // when cg_queue_destroy began (steady clock)
  QMetrics m;

  static constexpr uint32_t DEPTH = 2;  // batches per submitter: one running, the next queued

  // cg_queue_destroy waits this long for the device to drain what was dealt, then fails the rest
  // (CEDARGPU_QUEUE_STOP_GRACE_MS when the destroy begins, default 2000): a hung GPU cannot block
  // shutdown forever
  std::atomic<int64_t> grace_ns{2000000000};
  int64_t stop_grace_ns() const { return grace_ns.load(); }
  bool stopping_too_long() const;
  void fail_backlog(std::deque<std::shared_ptr<Ticket>>& backlog);

  void run();
  void work(QWorker& w);
  void publish(QBatch& qb) {
    for (auto& t : qb.tickets) t->ready.store(1, std::memory_order_release);
    qb.tickets.clear();  // breaks the ticket <-> batch reference cycle
    pub.fetch_add(1, std::memory_order_release);
    futex_wake_all(&pub);
  }
};

bool cg_queue::stopping_too_long() const {
  const int64_t t = stop_ns.load();
  return t && now_ns() - t > stop_grace_ns();
}

void cg_queue::fail_backlog(std::deque<std::shared_ptr<Ticket>>& backlog) {
  auto qb = std::make_shared<QBatch>();
  qb->rc = CG_E_STATE;
  qb->err = "queue closed before the request reached a device";
  for (auto& t : backlog) {
    uint32_t st = T_QUEUED;
    if (t->state.compare_exchange_strong(st, T_TAKEN)) { t->qb = qb; qb->tickets.push_back(t); }
  }
  backlog.clear();
  publish(*qb);
}

void cg_queue::work(QWorker& w) {
  // Pipelined: a batch dealt while the previous one runs is submitted before that one is waited
  // for, so its host side (string table, pinned staging, launch) overlaps the device work and its
  // upload queues right behind the previous batch's results on the context's stream.
  std::shared_ptr<QBatch> inflight;  // submitted, not yet waited for
  Clock::time_point busy_since{};    // device-busy accounting: the union of in-flight intervals
  auto finish = [&](std::shared_ptr<QBatch>& qb) {
    if (!qb->rc) {
      // no deadline while the queue runs; once it is closing, at most its grace (a hung device
      // then fails the batch's callers and cg_queue_destroy returns). The download is polled in
      // 10 ms slices even while running, so a close that begins during a wait on a hung device is
      // seen; host re-runs after it get the rest of the grace (none while running).
      int rc;
      for (;;) {
        const int64_t t = stop_ns.load();
        rc = cg::batch_wait(qb->b, now_ns() + 10000000, t ? t + stop_grace_ns() : -1);
        if (rc != CG_E_TIMEOUT || qb->b->downloaded || stopping_too_long()) break;
      }
      if (rc) {
        qb->rc = rc;
        qb->err = rc == CG_E_TIMEOUT ? std::string("queue closed while the device had not finished the batch") : qb->b->err;
      }
    }
    const auto now = Clock::now();
    device_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(now - busy_since).count();
    busy_since = now;
    w.n_batches++;
    w.n_requests += qb->b->items.size();
    const uint64_t bl = (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(now - qb->t_submit).count();
    m.blat[lat_bucket(bl)].fetch_add(1, std::memory_order_relaxed);
    m.blat_sum.fetch_add(bl, std::memory_order_relaxed);
    publish(*qb);
    {
      std::lock_guard<std::mutex> g(slot_mu);
      w.load.fetch_sub(1);
    }
    slot_cv.notify_one();
    qb.reset();
  };
  for (;;) {
    std::shared_ptr<QBatch> qb;
    {
      std::unique_lock<std::mutex> g(w.mu);
      if (!inflight) {
        w.cv.wait(g, [&] { return w.stop || !w.q.empty(); });
        if (w.q.empty()) return;  // stopped and drained
      }
      if (!w.q.empty()) {
        qb = std::move(w.q.front());
        w.q.pop_front();
      }
    }
    if (qb) {
      qb->t_submit = Clock::now();
      if (!inflight) busy_since = qb->t_submit;
      if (!qb->rc) {
        const int rc = cg_batch_submit(qb->b);
        if (rc) {
          qb->rc = rc;
          qb->err = qb->b->err;
        }
      }
    }
    if (inflight) finish(inflight);  // the previous batch's results, while the next one runs
    if (qb) {
      if (qb->rc) finish(qb);  // not submitted: its callers get the error now
      else inflight = std::move(qb);
    }
  }
}

void cg_queue::run() {
  std::deque<std::shared_ptr<Ticket>> backlog;  // drained, not yet batched (over max_batch, or another image)
  std::vector<std::shared_ptr<Ticket>> grab;
  auto drain = [&] {
    for (auto& st : stripes) {
      {
        std::lock_guard<std::mutex> g(st.mu);
        if (st.q.empty()) continue;
        grab.swap(st.q);
      }
      pending.fetch_sub((uint32_t)grab.size(), std::memory_order_relaxed);
      for (auto& t : grab) backlog.push_back(std::move(t));
      grab.clear();
    }
  };
  uint32_t rr = 0;  // round-robin start: ties (idle GPUs) take turns
  auto least = [&]() -> QWorker* {
    const uint32_t n = (uint32_t)workers.size();
    QWorker* best = workers[rr % n].get();
    for (uint32_t k = 1; k < n; k++) {
      QWorker* w = workers[(rr + k) % n].get();
      if (w->load.load() < best->load.load()) best = w;
    }
    return best;
  };
  for (;;) {
    drain();
    if (backlog.empty()) {
      if (stop.load()) return;
      pending.wait(0, std::memory_order_acquire);
      continue;
    }
    if (max_delay.count() > 0) {  // let the batch fill, counted from its first request
      const auto until = backlog.front()->t + max_delay;
      while (backlog.size() < max_batch && Clock::now() < until && !stop.load()) {
        std::this_thread::sleep_for(std::chrono::microseconds(20));
        drain();
      }
    }
    // a submitter with room; while every one has a batch running and one queued, keep draining
    // (the next batch grows)
    QWorker* w = least();
    while (w->load.load() >= DEPTH && !stopping_too_long()) {
      {
        std::unique_lock<std::mutex> g(slot_mu);
        // every submitter notifies when it frees a slot; the timeout only bounds a missed wake
        // (system_clock: pthread_cond_timedwait, which the thread sanitizer models)
        slot_cv.wait_until(g, std::chrono::system_clock::now() + std::chrono::microseconds(50),
                           [&] { return least()->load.load() < DEPTH; });
      }
      drain();
      w = least();
    }
    // the batch's image on that context: the encoding image's epoch (else the first context)
    const std::shared_ptr<LoadedImage> enc = backlog.front()->img;
    std::shared_ptr<LoadedImage> img = enc;
    if (w->ctx != ctxs[0]) {
      std::lock_guard<std::mutex> g(w->ctx->mu);
      auto it = w->ctx->images.find(enc->host->epoch);
      if (it != w->ctx->images.end()) img = it->second;
    }
    if (img == enc && w->ctx != ctxs[0]) w = workers[0].get();
    if (stopping_too_long()) {  // closing over a device that does not drain: fail what is left
      fail_backlog(backlog);
      return;
    }
    auto qb = std::make_shared<QBatch>();
    qb->b = new cg_batch();
    qb->b->ctx = w->ctx;
    qb->b->img = img;
    qb->b->host.img = img->host;
    while (!backlog.empty() && qb->b->items.size() < max_batch && backlog.front()->img == enc) {
      std::shared_ptr<Ticket> t = std::move(backlog.front());
      backlog.pop_front();
      uint32_t st = T_QUEUED;
      if (!t->state.compare_exchange_strong(st, T_TAKEN)) {  // its caller already returned
        n_abandoned++;
        continue;
      }
      try {
        qb->b->host.append(t->e);
        qb->b->items.push_back({(int32_t)qb->b->host.n() - 1, -1});
        t->qb = qb;
        t->idx = (uint32_t)qb->b->items.size() - 1;
      } catch (const std::exception& ex) {
        t->rc = CG_E_ARG;
        t->err = ex.what();
      }
      qb->tickets.push_back(std::move(t));
    }
    n_batches++;
    const uint64_t n = qb->b->items.size();
    m.bsize[size_bucket(n)].fetch_add(1, std::memory_order_relaxed);
    for (uint64_t m = max_seen.load(); n > m && !max_seen.compare_exchange_weak(m, n);) {
    }
    rr++;
    w->load.fetch_add(1);
    {
      std::lock_guard<std::mutex> g(w->mu);
      w->q.push_back(std::move(qb));
    }
    w->cv.notify_one();
  }
}

namespace {

std::shared_ptr<LoadedImage> active_image(cg_ctx* ctx, std::string& err) {
  std::lock_guard<std::mutex> g(ctx->mu);
  if (!ctx->active) err = "no active image";
  return ctx->active;
}

thread_local uint32_t t_stripe = 0xFFFFFFFFu;
thread_local std::string t_err;

// Hands the ticket to the flusher and sleeps until its batch is published, or until the deadline
// (steady-clock ns, < 0 none) passes: CG_E_TIMEOUT, the ticket stays with the flusher.
int wait_ticket(cg_queue* q, const TicketP& tp, int64_t deadline, std::string& err) {
  if (q->stop.load()) { err = "queue closed"; return CG_E_STATE; }
  if (deadline >= 0 && now_ns() >= deadline) { err = "deadline exceeded before the request was queued"; return CG_E_TIMEOUT; }
  if (t_stripe == 0xFFFFFFFFu) t_stripe = q->next_stripe.fetch_add(1) % STRIPES;
  Ticket& t = *tp;
  t.t = Clock::now();
  {
    Stripe& st = q->stripes[t_stripe];
    std::lock_guard<std::mutex> g(st.mu);
    st.q.push_back(tp);
  }
  if (q->pending.fetch_add(1, std::memory_order_release) == 0) q->pending.notify_one();
  for (;;) {
    const uint32_t w = q->pub.load(std::memory_order_acquire);
    if (t.ready.load(std::memory_order_acquire)) break;
    int64_t rel = -1;
    if (deadline >= 0) {
      rel = deadline - now_ns();
      if (rel <= 0) {
        uint32_t st = T_QUEUED;  // still queued: the flusher will drop it rather than batch it
        (void)t.state.compare_exchange_strong(st, T_ABANDONED);
        err = "deadline exceeded waiting for the device batch";
        return CG_E_TIMEOUT;
      }
    }
    futex_wait(&q->pub, w, rel);
  }
  if (t.rc) { err = t.err; return t.rc; }
  if (t.qb->rc) { err = t.qb->err; return t.qb->rc; }
  return CG_OK;
}

int put_string(const std::string& s, char* buf, size_t cap, size_t* need) {
  if (need) *need = s.size() + 1;
  if (!buf) return CG_OK;
  if (cap < s.size() + 1) return CG_E_RANGE;
  std::memcpy(buf, s.c_str(), s.size() + 1);
  return CG_OK;
}

// Queues the caller's encoded request, waits for its batch and renders the caller's result
// (authz: cg_batch_authz's Decision + reason; else cg_batch_decision + diagnostic).
int submit_ticket(cg_queue* q, const TicketP& tp, int64_t deadline, int* out, char* buf, size_t cap, size_t* need,
                  bool authz) {
  int rc = wait_ticket(q, tp, deadline, t_err);
  if (rc) return rc;
  const Ticket& t = *tp;
  q->n_requests++;
  cg_batch* b = t.qb->b;
  if (authz) {
    rc = cg_batch_authz(b, t.idx, out, buf, cap, need);
    if (rc && rc != CG_E_RANGE) t_err = b->err;
    return rc;
  }
  if ((rc = cg_batch_decision(b, t.idx, out, nullptr))) { t_err = b->err; return rc; }
  if (!buf && !need) return CG_OK;
  return cg_batch_diagnostic(b, t.idx, 0, buf, cap, need);
}

}  // namespace

extern "C" {

int cg_queue_create_multi(cg_ctx* const* ctxs, uint32_t n_ctx, uint32_t max_batch, uint32_t max_delay_us, cg_queue** out) {
  if (!ctxs || !n_ctx || !out || max_batch == 0) return CG_E_ARG;
  for (uint32_t k = 0; k < n_ctx; k++)
    if (!ctxs[k]) return CG_E_ARG;
  *out = nullptr;
  auto* q = new (std::nothrow) cg_queue();
  if (!q) return CG_E_ARG;
  q->ctxs.assign(ctxs, ctxs + n_ctx);
  q->max_batch = max_batch;
  q->max_delay = std::chrono::microseconds(max_delay_us);
  try {
    for (uint32_t k = 0; k < n_ctx; k++) {
      q->workers.push_back(std::make_unique<QWorker>());
      q->workers.back()->ctx = ctxs[k];
    }
    for (auto& w : q->workers) {
      QWorker* wp = w.get();
      w->th = std::thread([q, wp] { q->work(*wp); });
    }
    q->flusher = std::thread([q] { q->run(); });
  } catch (...) {
    for (auto& w : q->workers) {
      { std::lock_guard<std::mutex> g(w->mu); w->stop = true; }
      w->cv.notify_one();
      if (w->th.joinable()) w->th.join();
    }
    delete q;
    return CG_E_ARG;
  }
  *out = q;
  return CG_OK;
}

int cg_queue_create(cg_ctx* ctx, uint32_t max_batch, uint32_t max_delay_us, cg_queue** out) {
  return cg_queue_create_multi(&ctx, ctx ? 1u : 0u, max_batch, max_delay_us, out);
}

void cg_queue_destroy(cg_queue* q) {
  if (!q) return;
  if (const char* e = std::getenv("CEDARGPU_QUEUE_STOP_GRACE_MS")) q->grace_ns.store((int64_t)std::max(0LL, std::atoll(e)) * 1000000);
  q->stop_ns.store(now_ns());
  q->stop.store(true);
  q->pending.fetch_add(1);  // wakes the flusher, which deals what it holds and returns
  q->pending.notify_one();
  if (q->flusher.joinable()) q->flusher.join();
  for (auto& w : q->workers) {  // each submitter runs what it was dealt, then returns
    { std::lock_guard<std::mutex> g(w->mu); w->stop = true; }
    w->cv.notify_one();
    if (w->th.joinable()) w->th.join();
  }
  delete q;
}

int cg_queue_gpu_stats(cg_queue* q, uint32_t k, uint64_t* batches, uint64_t* requests) {
  if (!q || k >= q->workers.size()) return CG_E_ARG;
  if (batches) *batches = q->workers[k]->n_batches.load();
  if (requests) *requests = q->workers[k]->n_requests.load();
  return CG_OK;
}

const char* cg_queue_last_error(void) { return t_err.c_str(); }

namespace {

// One SubjectAccessReview body on the caller's thread: GetAuthorizerAttributes, Authorize's fast
// paths and RecordToCedarResource into t.e (returns 1), or a fast-path decision (returns 2, *fast
// and *reason set), or a CG_E_* error (< 0, t_err set).
int encode_sar(const LoadedImage& li, const char* sar_json, size_t len, Ticket& t, int* fast, std::string& reason) {
  EncodedRequest& e = t.e;
  int d = 0;
  *fast = -1;
  GUARD(t_err, { d = encode_sar_direct(*li.host, sar_json, len, e, *fast, reason); })
  if (d == 2) return 2;
  if (d == 0) {  // the general path: JSON tree, Attributes, entities
    std::vector<EntityIn> ents;
    RequestIn req;
    GUARD(t_err, {
      JVal v = json_parse(sar_json, len);
      Attributes a = attributes_from_sar(v);
      *fast = authorize_fast_path(a, reason);
      if (*fast >= 0) return 2;
      record_to_cedar(a, ents, req);
      encode_request(*li.host, ents, req, e);
    })
  }
  return 1;
}

int authorize_sar(cg_queue* q, const char* sar_json, size_t len, int64_t timeout_ns, int* decision, char* reason,
                  size_t cap, size_t* need) {
  const int64_t deadline = timeout_ns < 0 ? -1 : now_ns() + timeout_ns;
  TicketP tp = std::make_shared<Ticket>();
  Ticket& t = *tp;
  t.img = active_image(q->ctxs[0], t_err);
  if (!t.img) return CG_E_STATE;
  std::string r;
  const int d = encode_sar(*t.img, sar_json, len, t, decision, r);
  if (d < 0) return d;
  if (d == 2) {
    q->n_fast++;
    return put_string(r, reason, cap, need);
  }
  return submit_ticket(q, tp, deadline, decision, reason, cap, need, true);
}

// cg_queue_authorize_sar_n: the n requests encoded on the caller's thread, queued under one stripe
// lock, one sleep until every one's batch is published, then rendered into `out`.
int authorize_sar_n(cg_queue* q, const char* const* sars, const size_t* lens, uint32_t n, int64_t timeout_ns,
                    int* decisions, char* out, size_t cap, size_t* offsets, size_t* need) {
  const int64_t deadline = timeout_ns < 0 ? -1 : now_ns() + timeout_ns;
  std::shared_ptr<LoadedImage> img = active_image(q->ctxs[0], t_err);
  if (!img) return CG_E_STATE;
  std::vector<TicketP> tps(n);
  std::vector<std::string> fast_reason(n);
  std::vector<TicketP> queued;
  queued.reserve(n);
  for (uint32_t k = 0; k < n; k++) {
    tps[k] = std::make_shared<Ticket>();
    tps[k]->img = img;
    const int d = encode_sar(*img, sars[k], lens[k], *tps[k], &decisions[k], fast_reason[k]);
    if (d < 0) return d;
    if (d == 2) {
      q->n_fast++;
      tps[k].reset();
    } else {
      queued.push_back(tps[k]);
    }
  }
  if (!queued.empty()) {
    if (q->stop.load()) { t_err = "queue closed"; return CG_E_STATE; }
    if (t_stripe == 0xFFFFFFFFu) t_stripe = q->next_stripe.fetch_add(1) % STRIPES;
    const auto t0 = Clock::now();
    {
      Stripe& st = q->stripes[t_stripe];
      std::lock_guard<std::mutex> g(st.mu);
      for (auto& tp : queued) {
        tp->t = t0;
        st.q.push_back(tp);
      }
    }
    if (q->pending.fetch_add((uint32_t)queued.size(), std::memory_order_release) == 0) q->pending.notify_one();
    for (size_t left = 0;;) {  // every queued request's batch published (or the deadline)
      const uint32_t w = q->pub.load(std::memory_order_acquire);
      while (left < queued.size() && queued[left]->ready.load(std::memory_order_acquire)) left++;
      if (left == queued.size()) break;
      int64_t rel = -1;
      if (deadline >= 0) {
        rel = deadline - now_ns();
        if (rel <= 0) {
          for (auto& tp : queued) {
            uint32_t s0 = T_QUEUED;
            (void)tp->state.compare_exchange_strong(s0, T_ABANDONED);
          }
          t_err = "deadline exceeded waiting for the device batch";
          return CG_E_TIMEOUT;
        }
      }
      futex_wait(&q->pub, w, rel);
    }
    for (auto& tp : queued) {
      if (tp->rc) { t_err = tp->err; return tp->rc; }
      if (tp->qb->rc) { t_err = tp->qb->err; return tp->qb->rc; }
    }
  }
  // the reasons, NUL-terminated, side by side in `out` (offsets[k]: request k's)
  size_t pos = 0;
  std::vector<char> buf(4096);
  for (uint32_t k = 0; k < n; k++) {
    const char* r = nullptr;
    size_t rl = 0;
    if (!tps[k]) {
      r = fast_reason[k].c_str();
      rl = fast_reason[k].size();
    } else {
      const Ticket& t = *tps[k];
      q->n_requests++;
      size_t nd = 0;
      int rc = cg_batch_authz(t.qb->b, t.idx, &decisions[k], buf.data(), buf.size(), &nd);
      if (rc == CG_E_RANGE) {
        buf.resize(nd);
        rc = cg_batch_authz(t.qb->b, t.idx, &decisions[k], buf.data(), buf.size(), &nd);
      }
      if (rc) { t_err = t.qb->b->err; return rc; }
      r = buf.data();
      rl = nd ? nd - 1 : 0;
    }
    if (offsets) offsets[k] = pos;
    if (out && pos + rl + 1 <= cap) std::memcpy(out + pos, r, rl + 1);
    pos += rl + 1;
  }
  if (need) *need = pos;
  return (out && pos > cap) ? CG_E_RANGE : CG_OK;
}

int is_authorized_json(cg_queue* q, const char* item_json, size_t len, int64_t timeout_ns, int* allow, char* diag,
                       size_t cap, size_t* need) {
  const int64_t deadline = timeout_ns < 0 ? -1 : now_ns() + timeout_ns;
  std::vector<EntityIn> ents;
  RequestIn req;
  GUARD(t_err, {
    JVal v = json_parse(item_json, len);
    decode_json_item(v, ents, req);
  })
  TicketP tp = std::make_shared<Ticket>();
  Ticket& t = *tp;
  t.img = active_image(q->ctxs[0], t_err);
  if (!t.img) return CG_E_STATE;
  GUARD(t_err, { encode_request(*t.img->host, ents, req, t.e); })
  return submit_ticket(q, tp, deadline, allow, diag, cap, need, false);
}

// outcome index of a call (cg_queue_metrics.requests): the decision when it is valid; 4: not
// recorded (CG_E_RANGE: the caller repeats the call with room for the reason, which is the one
// counted)
uint32_t outcome(int rc, int d, bool admission) {
  if (rc == CG_E_RANGE) return 4u;
  if (rc != CG_OK) return 3u;
  if (admission) return d ? 1u : 0u;
  return (d >= 0 && d < 3) ? (uint32_t)d : 3u;
}

}  // namespace

int cg_queue_authorize_sar(cg_queue* q, const char* sar_json, size_t len, int64_t timeout_ns, int* decision,
                           char* reason, size_t cap, size_t* need) {
  if (!q || !sar_json || !decision) return CG_E_ARG;
  const auto t0 = Clock::now();
  const int rc = authorize_sar(q, sar_json, len, timeout_ns, decision, reason, cap, need);
  q->m.request(outcome(rc, *decision, false),
               (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now() - t0).count());
  return rc;
}

int cg_queue_authorize_sar_n(cg_queue* q, const char* const* sars, const size_t* lens, uint32_t n, int64_t timeout_ns,
                             int* decisions, char* reasons, size_t cap, size_t* offsets, size_t* need) {
  if (!q || (n && (!sars || !lens || !decisions))) return CG_E_ARG;
  const auto t0 = Clock::now();
  const int rc = authorize_sar_n(q, sars, lens, n, timeout_ns, decisions, reasons, cap, offsets, need);
  const uint64_t ns = (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now() - t0).count();
  for (uint32_t k = 0; k < n; k++) q->m.request(outcome(rc, rc ? 0 : decisions[k], false), ns);
  return rc;
}

int cg_queue_is_authorized_json(cg_queue* q, const char* item_json, size_t len, int64_t timeout_ns, int* allow,
                                char* diag, size_t cap, size_t* need) {
  if (!q || !item_json || !allow) return CG_E_ARG;
  const auto t0 = Clock::now();
  const int rc = is_authorized_json(q, item_json, len, timeout_ns, allow, diag, cap, need);
  q->m.request(outcome(rc, *allow, true),
               (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now() - t0).count());
  return rc;
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

const uint64_t* cg_metrics_latency_bounds(uint32_t* n) {
  if (n) *n = CG_LAT_BOUNDS;
  return k_lat_bounds;
}

int cg_queue_metrics_get(cg_queue* q, cg_queue_metrics* out, size_t size) {
  if (!q || !out || size != sizeof(cg_queue_metrics)) return CG_E_ARG;
  std::memset(out, 0, sizeof(*out));
  auto rd = [](const std::atomic<uint64_t>& x) { return x.load(std::memory_order_relaxed); };
  for (uint32_t o = 0; o < 4; o++) {
    out->requests[o] = rd(q->m.req[o]);
    for (uint32_t b = 0; b <= CG_LAT_BOUNDS; b++) out->latency[o][b] = rd(q->m.lat[o][b]);
    out->latency_sum_ns[o] = rd(q->m.lat_sum[o]);
  }
  out->fast = rd(q->n_fast);
  out->batches = rd(q->n_batches);
  for (uint32_t b = 0; b <= CG_BATCH_BUCKETS; b++) out->batch_size[b] = rd(q->m.bsize[b]);
  for (uint32_t b = 0; b <= CG_LAT_BOUNDS; b++) out->batch_latency[b] = rd(q->m.blat[b]);
  out->batch_latency_sum_ns = rd(q->m.blat_sum);
  out->abandoned = rd(q->n_abandoned);
  cg_ctx* c = q->ctxs[0];
  {
    std::lock_guard<std::mutex> g(c->mu);
    out->active_epoch = c->active ? c->active->host->epoch : 0;
  }
  out->activations = rd(c->activations);
  return CG_OK;
}

int cg_queue_dropped(cg_queue* q, uint64_t* abandoned) {
  if (!q || !abandoned) return CG_E_ARG;
  *abandoned = q->n_abandoned.load();
  return CG_OK;
}

// Load generator (bench support): `threads` caller threads issue `total` blocking
// cg_queue_authorize_sar calls, cycling over sars[0..n). Reports wall seconds, latency
// percentiles (ns) and decision counts (deny, allow, no opinion).
int cg_queue_loadgen(cg_queue* q, const char* const* sars, const size_t* lens, uint32_t n, uint32_t threads,
                     uint64_t total, double* seconds, uint64_t* lat_p50, uint64_t* lat_p99, uint64_t* lat_max,
                     uint64_t* counts) {
  return cg_queue_loadgen_n(q, sars, lens, n, threads, 1, total, seconds, lat_p50, lat_p99, lat_max, counts);
}

int cg_queue_loadgen_n(cg_queue* q, const char* const* sars, const size_t* lens, uint32_t n, uint32_t threads,
                       uint32_t per_call, uint64_t total, double* seconds, uint64_t* lat_p50, uint64_t* lat_p99,
                       uint64_t* lat_max, uint64_t* counts) {
  if (!q || !sars || !lens || !n || !threads || !per_call) return CG_E_ARG;
  std::atomic<uint64_t> next{0};
  std::atomic<int> first_rc{0};
  std::mutex err_mu;
  std::string first_err;
  std::vector<std::vector<uint64_t>> lat(threads);
  std::vector<std::array<uint64_t, 3>> cnt(threads, {0, 0, 0});
  auto work = [&](uint32_t t) {
    std::vector<char> buf(4096);
    std::vector<const char*> ps(per_call);
    std::vector<size_t> ls(per_call), offs(per_call);
    std::vector<int> ds(per_call);
    lat[t].reserve(total / threads + 1);
    for (uint64_t i; (i = next.fetch_add(per_call)) < total;) {
      const uint32_t m = (uint32_t)std::min<uint64_t>(per_call, total - i);
      for (uint32_t j = 0; j < m; j++) {
        const uint32_t k = (uint32_t)((i + j) % n);
        ps[j] = sars[k];
        ls[j] = lens[k];
      }
      size_t need = 0;
      const auto t1 = Clock::now();
      int rc;
      if (per_call == 1) {
        rc = cg_queue_authorize_sar(q, ps[0], ls[0], -1, &ds[0], buf.data(), buf.size(), &need);
        if (rc == CG_E_RANGE) {
          buf.resize(need);
          rc = cg_queue_authorize_sar(q, ps[0], ls[0], -1, &ds[0], buf.data(), buf.size(), &need);
        }
      } else {
        rc = cg_queue_authorize_sar_n(q, ps.data(), ls.data(), m, -1, ds.data(), buf.data(), buf.size(), offs.data(), &need);
        if (rc == CG_E_RANGE) {
          buf.resize(need);
          rc = cg_queue_authorize_sar_n(q, ps.data(), ls.data(), m, -1, ds.data(), buf.data(), buf.size(), offs.data(), &need);
        }
      }
      const uint64_t ns = (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now() - t1).count();
      for (uint32_t j = 0; j < m; j++) lat[t].push_back(ns);  // (each request's latency is its call's)
      if (rc) {
        int z = 0;
        if (first_rc.compare_exchange_strong(z, rc)) {
          std::lock_guard<std::mutex> g(err_mu);
          first_err = t_err;  // the worker's thread-local error, handed to the caller below
        }
        next = total;  // stop every worker
        return;
      }
      for (uint32_t j = 0; j < m; j++)
        if (ds[j] >= 0 && ds[j] < 3) cnt[t][(size_t)ds[j]]++;
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
