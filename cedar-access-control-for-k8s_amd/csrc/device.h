// Device bridge (implemented in cedar_eval.hip). Plain C++ declarations: no HIP types leak into the
// host engine or the C-ABI.
#pragma once
#include <cstddef>
#include <cstdint>
#include <memory>
#include <vector>

namespace cg {

struct Image;
struct Batch;

enum FuKind : uint32_t { FU_BIG = 0, FU_OVF = 1, FU_GEN = 2, FU_KINDS = 3 };

struct DevImage {
  int device = -1;
  uint32_t *pstream = nullptr, *tier_cend = nullptr, *chunks = nullptr, *cpool = nullptr, *gstr_off = nullptr, *hot = nullptr;
  uint32_t* act = nullptr;
  uint32_t *btab = nullptr, *bfilt = nullptr, *bstream = nullptr;  // scope index
  void* btab_mem = nullptr;  // the slot table btab points to (built at load from the entry list)
  uint32_t *srows = nullptr, *shash = nullptr;                      // static entities
  uint32_t *sctx = nullptr, *sbits = nullptr, *svals = nullptr;     // scope bitsets
  uint32_t* sbloom = nullptr;                                        // their context filter
  uint32_t sctx_mask = 0, sbits_words = 0, l2_vmask = 0, l2_lmask = 0;
  uint32_t n_kent = 0;  // key entities (Image::key_ents): valid key-entity indices are below it
  uint8_t* gstr_bytes = nullptr;
  // the one device allocation holding the image's device region (image.h DevSection); the arrays
  // above point into it at (blob offset - origin)
  void* base = nullptr;
  uint64_t origin = 0, region = 0;  // blob offset of base[0]; region bytes (dev_end - dev_begin)
  // the whole blob is on the device (origin 0, blob_len bytes at base): a delta image can patch it
  // on the device (dev_blob_patch)
  uint64_t blob_len = 0;
  uint32_t n_static = 0, smask = 0;
  uint32_t lane_need = 0;  // lane-scratch words per request (> LANE_WORDS: the GLANE stream kernel)
  uint32_t cslot_mask = 0;  // rows carry element-hash / prefix-hash lists (Image::list_mask, image.h)
  uint32_t lslot_mask = 0, like_off = 0;  // like slots (Image::lslot_mask) and their row offset
  uint32_t cls_compact = 0;  // the host lists duplicate classes (Image::cls_off): one hit slot per class
  uint32_t n_pol = 0, n_tiers = 0, n_gstr = 0, n_hot = 0, n_act = 0, amask_ok = 0, has_bytecode = 1, indexed = 0, bmask = 0, fmask = 0, combo_mask = 0;
  size_t bytes = 0;
};

// Per-context cache of device and pinned host buffers (size classes), so that a batch costs no
// hipMalloc / hipFree (hipFree synchronises the device) and its copies run from pinned memory.
struct DevPool;

struct DevBatch {
  int device = -1;
  DevPool* pool = nullptr;
  // inputs: one device block (heap | rows | bstr_off | bstr_bytes | grouping keys), one copy
  uint32_t *heap = nullptr, *rows = nullptr, *req_idx = nullptr, *bstr_off = nullptr;
  uint8_t* bstr_bytes = nullptr;
  // results: one device block (res | reasons_f | reasons_p | errs | pos_of), one copy back. A
  // request's results sit at its position in the first pass's launch order: the grouped order of a
  // grouped batch (so that a wave's requests write neighbouring slots), else the request index.
  // pos_of[i] (grouped batches only; the gather kernel inverts ord into it) is request i's position.
  uint32_t *res = nullptr, *reasons_f = nullptr, *reasons_p = nullptr, *errs = nullptr, *pos_of = nullptr;
  // On-device follow-up (every batch size): right behind the first pass a gather kernel sorts the
  // requests it left unfinished (RF_OVERFLOW) into three worklists, and each worklist is
  // evaluated again on the device into its own results, all inside the result block, so one D2H
  // copy brings back both passes and the timed step holds every launch that decides a request:
  //   FU_BIG  more hits than the probe kernel stages (RF_BIG): its large-stage variant
  //   FU_OVF  reason / error lists longer than the first pass holds (exact counts known, <= 64
  //           hits): the probe kernel again with 64 reasons / 16 errors per entry
  //   FU_GEN  structural comparisons (RF_GENERAL) or any overflow of a non-indexed image: the
  //           policy-stream kernel
  // fu_cnt[k] = requests the gather found for worklist k (device-side; entries past fu[k].cap are
  // left to the host re-run). fu[k].cap == 0: worklist k off. fu_cnt[FU_KINDS]: requests whose
  // key-entity indices fall outside the image's (BAD_KIDX: encoded for another image; the scan
  // enumerates their keys instead and the batch fails with CG_E_DEVICE).
  uint32_t* fu_cnt = nullptr;
  struct FollowUp {
    uint32_t *ids = nullptr, *res = nullptr, *rf = nullptr, *rp = nullptr, *er = nullptr;
    uint32_t cap = 0, capr = 0, cape = 0;
  } fu[3];
  // split first pass: the index scan's bucket lists (cedar_eval.hip SCAN_*), device only: per
  // position its count word, per wave of 8 positions its list total and its list (the 8 requests'
  // buckets packed together, each tagged with its request's place in the wave)
  uint32_t* scan = nullptr;
  void* scan_blk = nullptr;
  size_t scan_cls = 0;
  // grouped batch (Batch::dev_group): the step's first pass runs in the order ord with the rows
  // copied into that order (grows), sorted on the device from the encoder's grouping keys (gkeys, an
  // input section) through gkeys2 / gvals and the sort's temp storage; everything but gkeys in one
  // pool block (group.hip)
  const uint32_t* gkeys = nullptr;
  uint32_t *ord = nullptr, *grows = nullptr, *gkeys2 = nullptr, *gvals = nullptr;
  void *grp_blk = nullptr, *grp_temp = nullptr;
  size_t grp_cls = 0, grp_temp_bytes = 0;
  uint32_t* lane = nullptr;  // per-request lane scratch (images with lane_need > LANE_WORDS)
  void* lane_blk = nullptr;
  size_t lane_cls = 0;
  uint32_t n = 0, capr = 0, cape = 0, row_words = 0;
  // a small batch of an indexed image (n <= dev_small_n()): the whole step is one launch of the
  // one-request-per-wave probe kernel (no scan lists, no gather, no follow-up launches; what its
  // lists cannot hold goes to the host re-run)
  bool small = false;
  bool stepped = false;  // the step ran once since the upload (later steps reset their counters)
  // small batches download the results up to the overflow slots (dl_bytes of out_bytes); the slots
  // a batch took follow once its counter is read (dev_download_finish)
  size_t dl_bytes = 0;
  // zero-copy results (small batches, CEDARGPU_ZERO_COPY=0 turns it off): the kernel writes res,
  // the reason / error lists and the overflow slots straight into the pinned block at zc_out
  // (behind the staged inputs); only the counters, which take device atomics and live in the input
  // block, come back by copy (to zc_cnt). No results copy and no second round trip for the slots.
  bool zc = false;
  uint8_t* zc_out = nullptr;
  uint32_t* zc_cnt = nullptr;
  // some inputs were copied straight from the host batch's pinned arrays (engine.h pinned_take):
  // until the stream drains, those arrays are kept alive by `keep` (set when the batch is retired)
  bool direct = false;
  std::shared_ptr<void> keep;
  size_t heap_words = 0, bytes = 0;
  void *in_blk = nullptr, *out_blk = nullptr, *stage = nullptr;  // pool blocks (device, device, pinned)
  size_t in_cls = 0, out_cls = 0, stage_cls = 0, out_bytes = 0;
  void* stream = nullptr;  // the stream the batch's work runs on
  void* done = nullptr;    // event after the result download (dev_download_async)
  bool pending = false;    // work enqueued on the batch's buffers not yet waited for
  int64_t wait_t0 = 0;     // when the first wait on `done` began (dev_now_ns; 0: not yet)
  // profiled batch (Batch::prof): timing events before the H2D copies, after them, after the step
  // and after the D2H copy (dev_batch_profile)
  void* pev[4] = {nullptr, nullptr, nullptr, nullptr};
};
// The device intervals of a profiled batch after its download: H2D copies, the step, the D2H copy
// (ms); false when the batch was not profiled.
bool dev_batch_profile(const DevBatch& b, float* h2d_ms, float* step_ms, float* d2h_ms);

// Batches of at most this many requests on an indexed image run as one launch (DevBatch::small);
// CEDARGPU_SMALL_N overrides (0: never).
uint32_t dev_small_n();
// All functions return 0 on success, or a negative CG_E_* code with dev_last_error() set.
const char* dev_last_error();
int dev_count(int* n);
int dev_select(int device);
int dev_synchronize(int device);
// Device copy of an image read from `blob` (Image::deserialize): the whole blob (the device region
// and, for delta images, the host part) in one allocation and one H2D copy.
int dev_image_upload(int device, const Image& img, const uint8_t* blob, DevImage* out);
// Device copy on `device` of an image already on another (or the same) device: one peer copy of
// the blob (xGMI between GPUs).
int dev_image_copy(int device, const Image& img, const DevImage& src, DevImage* out);
// Adopts `dev_blob`, the whole serialized blob already in device memory on `device` (hipMalloc'd,
// e.g. the buffer a broadcast wrote): the arrays point into it, and dev_image_free frees it.
int dev_image_adopt(int device, const Image& img, void* dev_blob, DevImage* out);
// Delta images (delta.cpp): builds on `device` a new blob of new_len bytes from the base image's
// device blob (base.blob_len > 0) and literal bytes. pieces: (dst, len, src) triples covering
// [0, new_len), each at most DL_PIECE bytes; src is a base-blob offset, or DL_LIT | an offset into
// lit; then the word fixups (word index, value) pairs. One H2D copy of pieces, fixups and
// literals, two kernel launches; *out receives the new device
// buffer (hipMalloc'd: dev_image_adopt takes it, else dev_free).
constexpr uint64_t DL_LIT = 1ull << 63;
constexpr uint64_t DL_PIECE = 64 * 1024;
int dev_blob_patch(int device, const DevImage& base, const uint64_t* pieces, size_t n_pieces, const uint8_t* lit,
                   size_t lit_len, const uint32_t* fix, size_t n_fix, size_t new_len, void** out);
void dev_free(int device, void* p);
// blob_sum (delta.h) of n bytes of device memory, computed on the device
int dev_blob_sum(int device, const void* p, size_t n, uint64_t* out);
// Copies n bytes of device memory on `device` to host memory (pinned staging, one copy).
int dev_to_host(int device, const void* src, size_t n, void* dst);
void dev_image_free(DevImage* d);
int dev_pool_create(int device, DevPool** out);
void dev_pool_destroy(DevPool* p);
// Uploads the batch's inputs (staged through a pinned block, one H2D copy) and zeroes its results.
int dev_batch_upload(int device, const Batch& b, DevBatch* out, void* stream, DevPool* pool);
void dev_batch_free(DevBatch* d);  // returns the blocks to the batch's pool
struct DevSubset;
// The same without waiting, for a batch (and the re-run jobs it holds) that a caller gives up on
// while its work may still run (a missed deadline, a hung device): the blocks return to the pool
// once the batch's stream has passed a host callback enqueued behind that work, and never while
// it may still write them. No wait at all, so a caller's deadline holds even on a hung GPU.
void dev_batch_retire(DevBatch* d, std::vector<DevSubset>& held);
// Evaluates every request of the batch into the batch's device result buffers (async on stream).
int dev_eval(const DevImage& img, DevBatch& b, void* stream);
// Re-evaluates the subset idx[0..n) with larger result capacities (probe 1: on the probe kernel,
// 2: on its large-stage variant, for an indexed image; 0: the stream kernel). Results are compact
// in subset order. _begin enqueues one subset's re-run on `stream` (several subsets enqueued back
// to back share one wait); _end waits for the stream and points `v` at the results in the job's
// pinned block, valid until dev_subset_release returns the job's blocks to the pool.
struct DevSubset {
  DevPool* pool = nullptr;
  void* stream = nullptr;
  void* done = nullptr;  // event after the job's D2H copy
  void *dblk = nullptr, *hblk = nullptr;
  size_t dcls = 0, hcls = 0;
  uint32_t n = 0, capr = 0, cape = 0;
  size_t o_res = 0, o_rf = 0, o_rp = 0, o_er = 0, total = 0;
};
struct SubsetView {
  const uint32_t *res = nullptr, *rf = nullptr, *rp = nullptr, *er = nullptr;
};
int dev_subset_begin(const DevImage& img, const DevBatch& b, const uint32_t* idx, uint32_t n, uint32_t capr,
                     uint32_t cape, int probe, void* stream, DevSubset* job);
// deadline_ns: steady-clock deadline (dev_now_ns() scale), < 0 none. Returns DEV_TIMEOUT past it
// (the job stays in flight and keeps its blocks; release it only after its stream drained).
int dev_subset_end(DevSubset* job, SubsetView* v, int64_t deadline_ns = -1);
void dev_subset_release(DevSubset* job);
int dev_download(DevBatch& b, Batch& host, void* stream);
// Enqueues the results' copy into the batch's pinned block right behind its evaluation and records
// an event, so that the next batch's upload and launch queue behind it without a host round trip.
int dev_download_async(DevBatch& b, void* stream);
// Waits for that event (until deadline_ns, < 0 none: DEV_TIMEOUT past it, the batch stays in
// flight) and points the host batch at the results in the pinned block.
constexpr int DEV_TIMEOUT = -6;  // CG_E_TIMEOUT
int64_t dev_now_ns();
int dev_download_finish(DevBatch& b, Batch& host, int64_t deadline_ns = -1);
// Fault injection (cg_ctx_inject_fault): enqueues a one-thread kernel that waits `us` microseconds
// of device wall clock on `stream` (a slow GPU), at most 2 s.
int dev_stall(int device, void* stream, uint64_t us);
int dev_stream_create(int device, void** stream);
void dev_stream_destroy(void* stream);
int dev_stream_sync(void* stream);
// bench support: times `iters` launches of the evaluation kernel on `stream` with HIP events
int dev_time_eval(const DevImage& img, DevBatch& b, uint32_t iters, void* stream, float* ms_total);
// The same with an event at each phase boundary of every step: ms_phase[STEP_PHASES] (summed over
// the iterations) and the steps' total. Phases: device grouping, index scan (the whole first pass
// when it is one kernel), candidate pass, follow-up gather, and the three follow-up worklists.
enum StepPhase : uint32_t { PH_GROUP = 0, PH_SCAN, PH_CAND, PH_GATHER, PH_FU_BIG, PH_FU_OVF, PH_FU_GEN, STEP_PHASES };
int dev_time_split(const DevImage& img, DevBatch& b, uint32_t iters, void* stream, float* ms_phase, float* ms_total);
// group.hip: the device grouping of a batch (a radix sort of the encoder's 32-bit grouping keys,
// rows copied into the new order)
uint32_t group_bits();
bool group_gather();  // the grouped rows are copied into order (else read through the order)
size_t group_temp_bytes(uint32_t n);
// (zero: zero_n words the step's later kernels count into, cleared by the grouping's first kernel
// instead of a fill launch of their own)
int group_enqueue(const uint32_t* keys, const uint32_t* rows, uint32_t n, uint32_t row_words, uint32_t* grows,
                  uint32_t* ord, uint32_t* keys2, uint32_t* vals, void* temp, size_t temp_bytes, void* stream,
                  uint32_t* zero = nullptr, uint32_t zero_n = 0);

}  // namespace cg
