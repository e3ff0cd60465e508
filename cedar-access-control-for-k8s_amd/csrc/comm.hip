// Policy hot-reload broadcast over RCCL (xGMI between the GPUs of a node).
//
// The decision path has no collective: every GPU evaluates its own request shard against its
// replica of the compiled image. On a reload (the reference swaps the *cedar.PolicySet at
// internal/server/store/directory.go:81 and verified_permissions.go:99, and mutates it in place
// at crd.go:62,85,102,114), rank `root` compiles the new image once and one ncclBroadcast ships the
// serialized blob straight into each GPU's image storage; each rank activates it as the new epoch.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/cedargpu.h"

struct cg_comm {
  int device = 0, nranks = 1, rank = 0;
  ncclComm_t nccl = nullptr;
  hipStream_t stream = nullptr;
  std::string err;
  bool aborted = false;  // a collective failed or timed out here: the communicator was aborted
};

static thread_local std::string g_comm_err;

// Waits for the comm stream's collectives with a deadline, polling RCCL's asynchronous error. On
// an error or past the deadline this rank aborts its communicator (ncclCommAbort): its own pending
// collective ends and its resources are released, instead of a rank blocking forever inside a
// broadcast a failed peer never joins. The communicator is unusable afterwards (recreate it).
static bool comm_wait(cg_comm* c, int64_t timeout_ms, std::string& why) {
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    const hipError_t q = hipStreamQuery(c->stream);
    if (q == hipSuccess) return true;
    ncclResult_t ae = ncclSuccess;
    (void)ncclCommGetAsyncError(c->nccl, &ae);
    const bool late = std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(timeout_ms);
    if (q != hipErrorNotReady || (ae != ncclSuccess && ae != ncclInProgress) || late) {
      why = q != hipErrorNotReady ? std::string("stream: ") + hipGetErrorString(q)
            : late                ? std::string("collective timed out")
                                  : std::string("RCCL: ") + ncclGetErrorString(ae);
      (void)ncclCommAbort(c->nccl);
      c->nccl = nullptr;
      c->aborted = true;
      return false;
    }
    std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
}
// An RCCL call that fails at enqueue may leave the communicator in an error state: abort it as a
// failed wait does, so that a later call reports CG_E_STATE at once instead of blocking in a
// collective until the timeout.
static void comm_abort(cg_comm* c) {
  if (c->aborted) return;
  if (c->nccl) (void)ncclCommAbort(c->nccl);
  c->nccl = nullptr;
  c->aborted = true;
}
static int64_t comm_timeout_ms() {
  static const int64_t t = [] { const char* e = std::getenv("CEDARGPU_COMM_TIMEOUT_MS"); return e ? (int64_t)std::atoll(e) : 60000; }();
  return t;
}

extern "C" {

int cg_comm_unique_id(uint8_t* out, size_t cap) {
  if (!out || cap < NCCL_UNIQUE_ID_BYTES) return CG_E_ARG;
  ncclUniqueId id;
  ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) { g_comm_err = ncclGetErrorString(r); return CG_E_DEVICE; }
  std::memcpy(out, id.internal, NCCL_UNIQUE_ID_BYTES);
  return CG_OK;
}

int cg_comm_create(int device, int nranks, int rank, const uint8_t* id, size_t len, cg_comm** out) {
  if (!out || !id || len < NCCL_UNIQUE_ID_BYTES || nranks < 1 || rank < 0 || rank >= nranks) return CG_E_ARG;
  *out = nullptr;
  auto* c = new (std::nothrow) cg_comm();
  if (!c) return CG_E_ARG;
  c->device = device; c->nranks = nranks; c->rank = rank;
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    g_comm_err = "hipSetDevice / hipStreamCreate failed";
    delete c;
    return CG_E_DEVICE;
  }
  ncclUniqueId uid;
  std::memcpy(uid.internal, id, NCCL_UNIQUE_ID_BYTES);
  ncclResult_t r = ncclCommInitRank(&c->nccl, nranks, uid, rank);
  if (r != ncclSuccess) {
    g_comm_err = ncclGetErrorString(r);
    (void)hipStreamDestroy(c->stream);
    delete c;
    return CG_E_DEVICE;
  }
  *out = c;
  return CG_OK;
}

void cg_comm_destroy(cg_comm* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->nccl) (void)ncclCommDestroy(c->nccl);  // (an aborted communicator is already released)
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

const char* cg_comm_last_error(cg_comm* c) { return c ? c->err.c_str() : g_comm_err.c_str(); }

// Collective: every rank calls it. On `root`, image/len are the compiled blob; elsewhere they are
// ignored. The blob goes to device memory once on the root (one H2D copy) and one ncclBroadcast
// writes it into a device buffer on every other rank (xGMI, RCCL's own pipelining, no per-piece
// host sync); each rank's buffer then becomes its image's device storage as is
// (cg_image_load_device: no re-upload), loaded as `epoch` and activated when activate != 0.
// Every rank but the root copies the blob back once for its host-side tables. *out_len
// (optional) receives the blob size. A failure leaves a rank's active image as it was: a rank that
// cannot allocate makes every rank fail before the blob moves (an all-reduce of readiness), and a
// decode error after the broadcast is local to its rank; no rank is left waiting in a collective.
int cg_broadcast_image(cg_ctx* ctx, cg_comm* c, int root, const void* image, size_t len, uint64_t epoch, int activate,
                       size_t* out_len) {
  if (!ctx || !c || root < 0 || root >= c->nranks) return CG_E_ARG;
  if (c->aborted || !c->nccl) { c->err = "communicator aborted by an earlier failure; recreate it"; return CG_E_STATE; }
  auto fail = [&](const std::string& m) { c->err = m; return CG_E_DEVICE; };
  std::string why;
  if (hipSetDevice(c->device) != hipSuccess) return fail("hipSetDevice failed");
  // the root's length, or 0 when it has no blob: every rank then stops after this first collective
  uint64_t n = (c->rank == root && image) ? (uint64_t)len : 0;
  uint64_t* dn = nullptr;
  if (hipMalloc((void**)&dn, 8) != hipSuccess) return fail("hipMalloc failed");
  ncclResult_t r = ncclSuccess;
  bool ok = hipMemcpy(dn, &n, 8, hipMemcpyHostToDevice) == hipSuccess &&
            (r = ncclBroadcast(dn, dn, 8, ncclUint8, root, c->nccl, c->stream)) == ncclSuccess &&
            comm_wait(c, comm_timeout_ms(), why) && hipMemcpy(&n, dn, 8, hipMemcpyDeviceToHost) == hipSuccess;
  if (!ok) {
    if (r != ncclSuccess) comm_abort(c);
    (void)hipFree(dn);
    return fail(std::string("length broadcast: ") + (why.empty() ? ncclGetErrorString(r) : why.c_str()));
  }
  if (n == 0) {
    (void)hipFree(dn);
    c->err = "the root has no image to broadcast";
    return CG_E_ARG;
  }
  // every rank allocates its receive buffer (the root also stages the blob into it), then all agree
  // (min over ranks) before the blob moves: a rank whose allocation failed makes every rank return
  // CG_E_DEVICE instead of leaving the others inside a broadcast it never joins
  void* buf = nullptr;
  uint64_t ready = hipMalloc(&buf, (size_t)n) == hipSuccess ? 1u : 0u;
  if (ready && c->rank == root && hipMemcpy(buf, image, (size_t)n, hipMemcpyHostToDevice) != hipSuccess) ready = 0;
  ok = hipMemcpy(dn, &ready, 8, hipMemcpyHostToDevice) == hipSuccess &&
       (r = ncclAllReduce(dn, dn, 1, ncclUint64, ncclMin, c->nccl, c->stream)) == ncclSuccess &&
       comm_wait(c, comm_timeout_ms(), why) && hipMemcpy(&ready, dn, 8, hipMemcpyDeviceToHost) == hipSuccess;
  (void)hipFree(dn);
  if (r != ncclSuccess) comm_abort(c);
  if (!ok || !ready) {
    if (buf) (void)hipFree(buf);
    return fail(!ok ? std::string("readiness all-reduce: ") + (why.empty() ? ncclGetErrorString(r) : why.c_str())
                    : std::string("a rank could not allocate or stage the image buffer"));
  }
  // a failure from here on (RCCL error, dead peer, timeout) aborts this rank's communicator
  r = ncclBroadcast(buf, buf, (size_t)n, ncclUint8, root, c->nccl, c->stream);
  if (r != ncclSuccess || !comm_wait(c, comm_timeout_ms(), why)) {
    if (r != ncclSuccess) comm_abort(c);
    (void)hipFree(buf);
    return fail(std::string("image broadcast: ") + (why.empty() ? ncclGetErrorString(r) : why.c_str()));
  }
  int rc = cg_image_load_device(ctx, buf, (size_t)n, epoch, c->rank == root ? image : nullptr);
  if (rc) {
    (void)hipFree(buf);
    c->err = cg_last_error(ctx);
    return rc;
  }
  if (activate && (rc = cg_image_activate(ctx, epoch))) { c->err = cg_last_error(ctx); return rc; }
  if (out_len) *out_len = (size_t)n;
  return CG_OK;
}

// Collective: a delta image (cg_image_delta against `base_epoch`, which every rank holds) from
// `root` to every rank, applied on each GPU (cg_image_load_delta) and loaded as `epoch`. Only the
// delta's bytes cross xGMI (a one-CRD edit of the 100k-policy C5 image: ~0.1 % of the full blob).
// A last all-reduce makes the ranks agree: `epoch` is activated (activate != 0) only when every
// rank applied the delta, and every rank then returns the same result.
int cg_broadcast_delta(cg_ctx* ctx, cg_comm* c, int root, uint64_t base_epoch, const void* delta, size_t len,
                       uint64_t epoch, int activate, size_t* out_len) {
  if (!ctx || !c || root < 0 || root >= c->nranks) return CG_E_ARG;
  if (c->aborted || !c->nccl) { c->err = "communicator aborted by an earlier failure; recreate it"; return CG_E_STATE; }
  auto fail = [&](const std::string& m) { c->err = m; return CG_E_DEVICE; };
  std::string why;
  if (hipSetDevice(c->device) != hipSuccess) return fail("hipSetDevice failed");
  uint64_t* dn = nullptr;
  if (hipMalloc((void**)&dn, 8) != hipSuccess) return fail("hipMalloc failed");
  // one 8-byte collective on the comm stream; false (communicator aborted on enqueue errors) on failure
  auto coll8 = [&](uint64_t& v, bool bcast) {
    ncclResult_t r = ncclSuccess;
    const bool ok = hipMemcpy(dn, &v, 8, hipMemcpyHostToDevice) == hipSuccess &&
                    (r = bcast ? ncclBroadcast(dn, dn, 8, ncclUint8, root, c->nccl, c->stream)
                               : ncclAllReduce(dn, dn, 1, ncclUint64, ncclMin, c->nccl, c->stream)) == ncclSuccess &&
                    comm_wait(c, comm_timeout_ms(), why) && hipMemcpy(&v, dn, 8, hipMemcpyDeviceToHost) == hipSuccess;
    if (r != ncclSuccess) {
      comm_abort(c);
      why = ncclGetErrorString(r);
    }
    return ok;
  };
  uint64_t n = (c->rank == root && delta) ? (uint64_t)len : 0;
  if (!coll8(n, true)) { (void)hipFree(dn); return fail("length broadcast: " + why); }
  if (n == 0) {
    (void)hipFree(dn);
    c->err = "the root has no delta to broadcast";
    return CG_E_ARG;
  }
  void* buf = nullptr;
  uint64_t ready = hipMalloc(&buf, (size_t)n) == hipSuccess ? 1u : 0u;
  if (ready && c->rank == root && hipMemcpy(buf, delta, (size_t)n, hipMemcpyHostToDevice) != hipSuccess) ready = 0;
  if (!coll8(ready, false) || !ready) {
    if (buf) (void)hipFree(buf);
    (void)hipFree(dn);
    return fail(!why.empty() ? "readiness all-reduce: " + why : std::string("a rank could not allocate the delta buffer"));
  }
  ncclResult_t r = ncclBroadcast(buf, buf, (size_t)n, ncclUint8, root, c->nccl, c->stream);
  if (r != ncclSuccess || !comm_wait(c, comm_timeout_ms(), why)) {
    if (r != ncclSuccess) comm_abort(c);
    (void)hipFree(buf);
    (void)hipFree(dn);
    return fail("delta broadcast: " + (why.empty() ? std::string(ncclGetErrorString(r)) : why));
  }
  std::vector<uint8_t> host;
  const void* hd = delta;
  int rc = CG_OK;
  if (c->rank != root) {
    host.resize((size_t)n);
    if (hipMemcpy(host.data(), buf, (size_t)n, hipMemcpyDeviceToHost) != hipSuccess) rc = CG_E_DEVICE;
    hd = host.data();
  }
  (void)hipFree(buf);
  std::string local;
  if (rc == CG_OK) {
    rc = cg_image_load_delta(ctx, base_epoch, hd, (size_t)n, epoch);
    if (rc) local = cg_last_error(ctx);
  } else {
    local = "D2H of the delta failed";
  }
  uint64_t all = rc == CG_OK ? 1u : 0u;
  if (!coll8(all, false)) { (void)hipFree(dn); return fail("result all-reduce: " + why); }
  (void)hipFree(dn);
  if (!all) {
    c->err = rc ? local : std::string("another rank could not apply the delta (epoch loaded here, not activated)");
    return rc ? rc : CG_E_STATE;
  }
  if (activate && (rc = cg_image_activate(ctx, epoch))) { c->err = cg_last_error(ctx); return rc; }
  if (out_len) *out_len = (size_t)n;
  return CG_OK;
}

}  // extern "C"
