// Policy hot-reload broadcast over RCCL (xGMI between the GPUs of a node).
//
// The decision path has no collective: every GPU evaluates its own request shard against its
// replica of the compiled image. On a reload (the reference swaps the *cedar.PolicySet at
// internal/server/store/directory.go:81 and verified_permissions.go:99, and mutates it in place
// at crd.go:62,85,102,114), rank `root` compiles the new image once and one ncclBroadcast ships the
// serialized blob to every GPU; each rank then loads and activates it as the new epoch.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <string>
#include <vector>

#include "../../include/cedargpu.h"

struct cg_comm {
  int device = 0, nranks = 1, rank = 0;
  ncclComm_t nccl = nullptr;
  hipStream_t stream = nullptr;
  std::string err;
};

static thread_local std::string g_comm_err;

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
  if (c->nccl) (void)ncclCommDestroy(c->nccl);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

const char* cg_comm_last_error(cg_comm* c) { return c ? c->err.c_str() : g_comm_err.c_str(); }

// Collective: every rank calls it. On `root`, image/len are the compiled blob; elsewhere they are
// ignored. The blob goes through one device buffer per rank; every rank then loads it into ctx as
// `epoch` (and activates it when activate != 0). *out_len (optional) receives the blob size.
int cg_broadcast_image(cg_ctx* ctx, cg_comm* c, int root, const void* image, size_t len, uint64_t epoch, int activate,
                       size_t* out_len) {
  if (!ctx || !c || root < 0 || root >= c->nranks) return CG_E_ARG;
  if (c->rank == root && !image) return CG_E_ARG;
  auto fail = [&](const std::string& m) { c->err = m; return CG_E_DEVICE; };
  if (hipSetDevice(c->device) != hipSuccess) return fail("hipSetDevice failed");
  uint64_t n = c->rank == root ? (uint64_t)len : 0;
  void* d = nullptr;
  const size_t cap = 1 << 20;
  if (hipMalloc(&d, cap) != hipSuccess) return fail("hipMalloc failed");
  std::vector<uint8_t> blob;
  int rc = CG_OK;
  do {
    // length first (8 bytes), then the blob in device-buffer-sized pieces
    if (hipMemcpy(d, &n, 8, hipMemcpyHostToDevice) != hipSuccess) { rc = fail("H2D failed"); break; }
    ncclResult_t r = ncclBroadcast(d, d, 8, ncclUint8, root, c->nccl, c->stream);
    if (r != ncclSuccess || hipStreamSynchronize(c->stream) != hipSuccess) { rc = fail(std::string("ncclBroadcast: ") + ncclGetErrorString(r)); break; }
    if (hipMemcpy(&n, d, 8, hipMemcpyDeviceToHost) != hipSuccess) { rc = fail("D2H failed"); break; }
    if (c->rank != root) blob.resize((size_t)n);
    const uint8_t* src = c->rank == root ? (const uint8_t*)image : nullptr;
    for (uint64_t off = 0; off < n && rc == CG_OK; off += cap) {
      const size_t piece = (size_t)std::min<uint64_t>(cap, n - off);
      if (c->rank == root && hipMemcpy(d, src + off, piece, hipMemcpyHostToDevice) != hipSuccess) { rc = fail("H2D failed"); break; }
      r = ncclBroadcast(d, d, piece, ncclUint8, root, c->nccl, c->stream);
      if (r != ncclSuccess || hipStreamSynchronize(c->stream) != hipSuccess) { rc = fail(std::string("ncclBroadcast: ") + ncclGetErrorString(r)); break; }
      if (c->rank != root && hipMemcpy(blob.data() + off, d, piece, hipMemcpyDeviceToHost) != hipSuccess) { rc = fail("D2H failed"); break; }
    }
  } while (0);
  (void)hipFree(d);
  if (rc) return rc;
  const void* img = c->rank == root ? image : (const void*)blob.data();
  if ((rc = cg_image_load(ctx, img, (size_t)n, epoch))) { c->err = cg_last_error(ctx); return rc; }
  if (activate && (rc = cg_image_activate(ctx, epoch))) { c->err = cg_last_error(ctx); return rc; }
  if (out_len) *out_len = (size_t)n;
  return CG_OK;
}

}  // extern "C"
