/* cedargpu — MI355X-native Cedar authorization for the cedar-access-control-for-k8s webhooks.
 *
 * C-ABI boundary (plain pointers and sizes; no C++ or HIP types cross it). It replaces, behind the
 * reference's own store interface, the per-request evaluation the reference performs with
 * cedar-go v1.1.0:
 *
 *   internal/server/store/store.go:9-15   PolicyStore.PolicySet() *cedar.PolicySet
 *   internal/server/store/store.go:25-42  TieredPolicyStores.IsAuthorized(EntityMap, Request)
 *                                         -> (cedar.Decision, cedar.Diagnostic)
 *   internal/server/store/store.go:31     (*cedar.PolicySet).IsAuthorized  (the hot path)
 *   internal/server/store/memory.go:18    cedar.NewPolicySetFromBytes       (IDs policy<i>)
 *   internal/server/store/directory.go:69 cedar.NewPolicyListFromBytes      (IDs <file>.policy<i>)
 *   internal/server/store/crd.go:51,60    per-CRD lists                     (IDs <name><i>-<uid>)
 *   internal/server/store/verified_permissions.go:89,95                     (IDs <id>.<i>)
 *   cmd/cedar-webhook/main.go:111-116     static allow-all-admission store
 *
 * Every call returns 0 (CG_OK) or a negative CG_E_* status; no exception crosses the boundary.
 * Strings in/out are UTF-8. See INTEGRATION.md for the cgo binding a maintainer would add.
 */
#ifndef CEDARGPU_H
#define CEDARGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CG_OK 0
#define CG_E_ARG (-1)      /* bad argument / malformed JSON */
#define CG_E_PARSE (-2)    /* Cedar syntax error (cedar.NewPolicySetFromBytes would fail) */
#define CG_E_COMPILE (-3)  /* valid Cedar the device compiler cannot lower */
#define CG_E_STATE (-4)    /* call out of order (no active image, batch not submitted, ...) */
#define CG_E_DEVICE (-5)   /* HIP runtime / kernel failure (callers fail safe: authz NoOpinion, admission allow) */
#define CG_E_TIMEOUT (-6)
#define CG_E_RANGE (-7)    /* index out of range / buffer too small (see *need) */

typedef struct cg_compiler cg_compiler;
typedef struct cg_ctx cg_ctx;
typedef struct cg_batch cg_batch;
typedef struct cg_comm cg_comm;

const char* cg_version(void);
void cg_free(void* p);

/* ---- compiler: policy documents -> serialized, versioned image (host only; no GPU needed) ---- */
int cg_compiler_create(cg_compiler** out);
void cg_compiler_destroy(cg_compiler* c);
const char* cg_compiler_last_error(cg_compiler* c);
/* Starts the next tier (one TieredPolicyStores element, store.go:20). */
int cg_compiler_add_tier(cg_compiler* c);
/* Adds every policy of a Cedar document to the current tier with IDs id_prefix + i + id_suffix:
 * memory store: ("policy", ""), directory: ("<file>.policy", ""), CRD: ("<name>", "-<uid>"),
 * AVP: ("<id>.", ""). `filename` becomes Position.filename. Documents are parsed by
 * cg_compiler_build; one that does not parse fails the build with CG_E_PARSE, as
 * cedar.NewPolicySetFromBytes fails NewMemoryStore (store/memory.go:17-22). */
int cg_compiler_add_document(cg_compiler* c, const char* filename, const char* text, size_t len,
                             const char* id_prefix, const char* id_suffix);
/* As cg_compiler_add_document; with CG_DOC_SKIP_INVALID a document that does not parse is left out
 * of the build (no policies) and listed by cg_compiler_doc_errors, while the build succeeds: the
 * directory, CRD and AVP stores log such a document and load the rest (store/directory.go:69-73,
 * crd.go:51-55 and 91-95 -- an update that breaks a CRD drops its old policies --,
 * verified_permissions.go:89-93). */
#define CG_DOC_SKIP_INVALID 1
int cg_compiler_add_document_ex(cg_compiler* c, const char* filename, const char* text, size_t len,
                                const char* id_prefix, const char* id_suffix, int flags);
/* The documents the last cg_compiler_build left out: JSON [{"filename":..,"error":..}, ...].
 * Writes at most cap bytes incl. NUL; *need = required size. */
int cg_compiler_doc_errors(cg_compiler* c, char* buf, size_t cap, size_t* need);
/* Adds exactly one policy with an explicit ID. zero_position=1 reproduces policies built from an
 * AST (cedar.NewPolicyFromAST, e.g. allow-all-admission) whose Position is the zero value. */
int cg_compiler_add_policy(cg_compiler* c, const char* policy_id, const char* filename, const char* text,
                           size_t len, int zero_position);
/* Sets the image's static entities: a JSON array of Cedar entities ({"uid":{"type","id"},
 * "attrs":{...},"parents":[...]}) such as a group / namespace hierarchy that the requests' EntityMaps
 * do not carry (the reference's SAR path gives groups no parents, internal/server/entities/
 * user.go:40-54; a deeper hierarchy, like store_test.go:35-40's user -> group edge, needs a static
 * source). Every evaluation then sees the request's EntityMap merged with them: a static entity the
 * request lacks is present; for a UID in both, the request's attributes and the union of both parent
 * lists. The compiler builds each static entity's transitive `in`-closure row into the image.
 * Replaces any earlier set; an empty array (len 0) clears it.
 * Limits of the device row format: an entity may have at most 65,535 transitive ancestors (request
 * parents and static closure together), at most 32,767 of them scope-index key entities; a request
 * past either is refused by the encoder with CG_E_PARSE / CG_E_COMPILE (never evaluated on a
 * truncated list). */
int cg_compiler_set_entities(cg_compiler* c, const char* json, size_t len);
/* Drops the tiers added so far but keeps the compiler's parse cache: the incremental rebuild after
 * a store change (a CRD added / updated / removed, crd.go:45-118; a directory re-read,
 * directory.go:41-82; an AVP sync, verified_permissions.go:58-100) re-adds every document and
 * parses only those whose (filename, text) the previous build did not have. */
int cg_compiler_clear(cg_compiler* c);
/* Documents the last build took from the parse cache / parsed anew, and cache entries kept. */
int cg_compiler_cache_stats(cg_compiler* c, uint64_t* hits, uint64_t* misses, uint64_t* entries);
/* Compiles all tiers into an image blob (free with cg_free). Unseen documents parse on worker
 * threads. A full build's blob is byte-identical to a build by a fresh compiler. After a full
 * build, a rebuild lowers only the documents the last build did not have (the per-event
 * PolicySet.Add / Remove of crd.go:62,85,102,114, applied to the lowered image instead of the AST)
 * and copies every other document's lowered policies: its image decides every request as a fresh
 * build would, but keeps the removed documents' words until the next full build (not byte-
 * identical). A rebuild is a full one when the image-wide choices changed (hot attribute paths,
 * an action table past 64 entries, the static entities) or the arenas hold more garbage than live
 * words. */
int cg_compiler_build(cg_compiler* c, uint64_t epoch, uint8_t** image, size_t* len);
/* The same build in two steps, for callers that own the blob's memory: cg_compiler_build_sized
 * compiles and holds the image, returning its blob size; cg_compiler_write_image serializes it into
 * the caller's buffer of at least that size (large sections copied on several threads) and drops
 * it. No intermediate copy of the blob (C5's 113 MB image). */
int cg_compiler_build_sized(cg_compiler* c, uint64_t epoch, size_t* len);
int cg_compiler_write_image(cg_compiler* c, void* out, size_t cap);
/* Incremental rebuilds on (default) or off (every build a full one). */
int cg_compiler_set_incremental(cg_compiler* c, int on);
/* The last build: *incremental 1 when it reused lowered documents, policies it lowered and reused,
 * and a full build's reason ("first build", "hot attribute paths changed", "compaction", ...). */
int cg_compiler_last_build(cg_compiler* c, int* incremental, uint64_t* lowered, uint64_t* reused, const char** why_full);
/* Number of policies / tiers of a built image blob. */
int cg_image_info(const void* image, size_t len, uint32_t* n_policies, uint32_t* n_tiers, uint64_t* epoch);
/* Compiled-image shape (no reference counterpart; diagnostics and tests): policies lowered to
 * predicate atoms (the rest run as bytecode), pre-resolved hot attributes, distinct action
 * entities in scopes, policy-stream words. */
int cg_image_stats(const void* image, size_t len, uint32_t* n_atomic, uint32_t* n_hot, uint32_t* n_actions,
                   uint32_t* stream_words);

/* Scope-index shape (diagnostics and tests): hot slots whose rows carry element-hash lists (sets a
 * contains / containsAny atom reads) and prefix-hash lists (`like "lit*"` keys), level-1 key combos
 * in use, index entries, and scope-bitset contexts x words per context row. */
int cg_image_index_stats(const void* image, size_t len, uint32_t* cslot_mask, uint32_t* pslot_mask,
                         uint32_t* combo_mask, uint32_t* entries, uint32_t* contexts, uint32_t* sbits_words);

/* Hot slots whose rows carry like words (Image::lslot_mask: each such slot's length and first / last
 * 8 bytes shipped in the request row, CEDARGPU_LIKE_WORDS=1 at compile time) and the slots any
 * `like` atom reads as bytes (Image::lread_mask). Host only; introspection for tests and tooling. */
int cg_image_like_slots(const void* image, size_t len, uint32_t* row_like_mask, uint32_t* like_read_mask);

/* 1 when policy i (image order) lowered to predicate atoms, 0 when it runs as bytecode. */
int cg_image_policy_atomic(const void* image, size_t len, uint32_t i, int* atomic);
/* 1 when the image is evaluated by the probe kernel over the scope index (all policies atomic). */
int cg_image_indexed(const void* image, size_t len, int* indexed);

/* ---- device context (one per GPU; requests shard across contexts, images are replicated) ---- */
int cg_device_count(int* n);
/* hipDeviceSynchronize on `device` (bench barriers; the library links ROCm's own HIP runtime). */
int cg_device_synchronize(int device);
int cg_ctx_create(int device, cg_ctx** out);
void cg_ctx_destroy(cg_ctx* ctx);
/* The context's last error; with ctx == NULL, the calling thread's last device error (why a
 * cg_ctx_create or cg_device_count failed). */
const char* cg_last_error(cg_ctx* ctx);
/* Gameday fault injection for the fail-safe path (the evaluator's counterpart of the reference's
 * ErrorInjector, internal/server/error_injector.go:11-50, gated there by
 * --confirm-non-prod-inject-errors; not for production). CG_FAULT_DEVICE_ERROR: the next `arg`
 * batch submits on ctx fail with CG_E_DEVICE without touching the device. CG_FAULT_STALL: every
 * batch submit first runs a device kernel that waits `arg` microseconds (at most 2 s), as a slow or
 * stuck GPU would. CG_FAULT_BAD_KIDX: the next `arg` batches carry principal key-entity indices the
 * image does not have, as a batch encoded for another image would; the device detects them (the
 * requests fall back to exact key enumeration) and cg_batch_wait fails the batch with CG_E_DEVICE.
 * CG_FAULT_NONE clears all. */
#define CG_FAULT_NONE 0
#define CG_FAULT_DEVICE_ERROR 1
#define CG_FAULT_STALL 2
#define CG_FAULT_BAD_KIDX 3
int cg_ctx_inject_fault(cg_ctx* ctx, int kind, uint64_t arg);
/* Diagnostics of the process-wide pinned pool the encoder writes small batches' arrays into:
 * bytes of pinned blocks held, blocks idle (free for the next batch), and batches that were closed
 * while their upload from those blocks could still run and so handed their arrays to the retired
 * batch until its stream drains. Any pointer may be NULL. (No reference counterpart: a test hook.) */
int cg_pinned_stats(uint64_t* held_bytes, uint64_t* idle_blocks, uint64_t* kept_batches);
/* Copies and uploads an image; the caller keeps ownership of `image`. Not active until activated. */
int cg_image_load(cg_ctx* ctx, const void* image, size_t len, uint64_t epoch);
/* Loads an image whose serialized blob is already in device memory on ctx's device, e.g. the
 * buffer a collective delivered it to (cg_broadcast_image): the blob's device region is used in
 * place (no copy); `host_blob` is the same bytes in host memory, or NULL to copy them back for the
 * host-side tables. dev_blob must come from hipMalloc on ctx's device; on success the library owns
 * it (hipFree when the image is dropped). The reference swaps its whole policy set on a reload
 * (directory.go:81, verified_permissions.go:99; crd.go:62-114 per CRD event). */
int cg_image_load_device(cg_ctx* ctx, void* dev_blob, size_t len, uint64_t epoch, const void* host_blob);
/* Loads onto `dst` the image `src` holds for `epoch`: the host tables are shared, the device region
 * is copied GPU to GPU (xGMI peer copy; a device copy when both contexts use the same GPU). The
 * in-process multi-GPU reload: compile once, cg_image_load on one context, this on the others. */
int cg_image_load_peer(cg_ctx* dst, cg_ctx* src, uint64_t epoch);
/* ---- delta images (src/delta.h) ----
 * A policy edit changes a few policies of a large image: the reference applies each CRD informer
 * event to its PolicySet in place (store/crd.go:45-118, mutations at :62,85,102,114). Here the root
 * compiles the new epoch (incrementally) and ships only the bytes that differ from the image every
 * GPU already holds. cg_image_delta: the delta that turns blob `base` into blob `next` (malloc'd,
 * cg_free). cg_image_patch: the new blob from base + delta on the host (checked against the delta's
 * checksum of the new blob; CG_E_ARG on any mismatch). cg_delta_info: a delta's sizes. */
int cg_image_delta(const void* base, size_t base_len, const void* next, size_t next_len, uint8_t** delta,
                   size_t* delta_len);
int cg_image_patch(const void* base, size_t base_len, const void* delta, size_t delta_len, uint8_t** out,
                   size_t* out_len);
int cg_delta_info(const void* delta, size_t len, uint64_t* base_len, uint64_t* new_len, uint64_t* ops,
                  uint64_t* literal_bytes);
/* Loads as `epoch` the image a delta makes of the image ctx holds for `base_epoch`: the new blob is
 * built on the GPU from the base's device copy (one copy kernel over the delta's operations), its
 * checksum checked, the host tables read from it. CG_E_STATE: no such base; CG_E_ARG: the delta is
 * malformed or for another base. Not active until activated. */
int cg_image_load_delta(cg_ctx* ctx, uint64_t base_epoch, const void* delta, size_t len, uint64_t epoch);
/* Atomically makes `epoch` the image new batches bind to; in-flight batches keep theirs. */
int cg_image_activate(cg_ctx* ctx, uint64_t epoch);
int cg_image_active(cg_ctx* ctx, uint64_t* epoch);
/* Drops a loaded image (no-op while batches still reference it; freed when the last one goes). */
int cg_image_unload(cg_ctx* ctx, uint64_t epoch);

/* ---- multi-GPU hot reload (RCCL over xGMI; no collective on the decision path) ----
 * Requests shard across GPUs, each holding a replica of the image. On a policy reload (the
 * reference swaps the PolicySet at store/directory.go:81, verified_permissions.go:99 and mutates it
 * at crd.go:62,85,102,114) one rank compiles and cg_broadcast_image ships the blob to every GPU.
 * cg_comm_unique_id: 128-byte RCCL id, made on one rank and shared out of band (cap >= 128). */
int cg_comm_unique_id(uint8_t* out, size_t cap);
int cg_comm_create(int device, int nranks, int rank, const uint8_t* id, size_t len, cg_comm** out);
void cg_comm_destroy(cg_comm* comm);
const char* cg_comm_last_error(cg_comm* comm);
/* Collective over comm: root's image (len bytes) is broadcast; every rank loads it into ctx as
 * `epoch` and activates it when activate != 0. *out_len (may be NULL) receives the blob size.
 * Failure keeps each rank's active image. A rank that cannot allocate makes every rank fail before
 * the blob moves; an RCCL error, a dead peer or a collective past CEDARGPU_COMM_TIMEOUT_MS (60 s)
 * aborts this rank's communicator (ncclCommAbort) and returns CG_E_DEVICE; later calls on it
 * return CG_E_STATE until it is recreated. */
int cg_broadcast_image(cg_ctx* ctx, cg_comm* comm, int root, const void* image, size_t len, uint64_t epoch,
                       int activate, size_t* out_len);
/* Collective: root's delta image against `base_epoch` (every rank holds it) is broadcast and applied
 * on every GPU (cg_image_load_delta) as `epoch`. The ranks agree on the outcome (a last all-reduce):
 * `epoch` is activated (activate != 0) only when every rank applied the delta. Failure handling as
 * cg_broadcast_image. *out_len (may be NULL) receives the delta's size. */
int cg_broadcast_delta(cg_ctx* ctx, cg_comm* comm, int root, uint64_t base_epoch, const void* delta, size_t len,
                       uint64_t epoch, int activate, size_t* out_len);

/* How request i of a waited batch was finished (introspection for tests and tooling): a bit set
 * of CG_ROUTE_*. 0: the first pass alone. FIRST_SLOT: the first pass wrote its long list into a
 * long-list worklist slot; FU_BIG / FU_OVF / FU_GEN: the large stage, the long-list follow-up or
 * the policy-stream follow-up on the device; RERUN: a host-driven re-run; CLASS: its reasons
 * include a duplicate class the device reported whole (its members listed on the host).
 * reason_words (optional): the deciding list's length as the device wrote it (a class reported
 * whole is one word; cg_batch_reasons lists its members). */
#define CG_ROUTE_FU_BIG 1u
#define CG_ROUTE_FU_OVF 2u
#define CG_ROUTE_FU_GEN 4u
#define CG_ROUTE_FIRST_SLOT 8u
#define CG_ROUTE_RERUN 16u
#define CG_ROUTE_CLASS 32u
int cg_batch_route(cg_batch* b, uint32_t i, uint32_t* route, uint32_t* reason_words);

/* ---- batches of (EntityMap, Request) ---- */
/* Creates a batch bound to the currently active image. */
int cg_batch_create(cg_ctx* ctx, cg_batch** out);
void cg_batch_destroy(cg_batch* b);
/* Appends requests: one JSON object {"entities":[<cedar entity json>...],"request":{"principal":
 * {"type","id"},"action":{...},"resource":{...},"context":{...}}} or a JSON array of them. */
int cg_batch_add_json(cg_batch* b, const char* json, size_t len);
uint32_t cg_batch_size(cg_batch* b);
/* Encodes strings, uploads the batch to the device and launches evaluation (asynchronous). */
int cg_batch_submit(cg_batch* b);
/* Waits for completion, binds the results and re-runs from the host what the device could not fit.
 * timeout_ns < 0: no deadline. Otherwise returns CG_E_TIMEOUT once timeout_ns has passed; a
 * timeout in the first wait leaves the batch in flight (wait again, or destroy it, which drains
 * its stream), a timeout during a host re-run fails the batch. Callers fail safe on CG_E_TIMEOUT
 * and CG_E_DEVICE as on a webhook timeout (mount/authorization-config.yaml:11,16 failurePolicy
 * NoOpinion; manifests/admission-webhook.yaml:11 failurePolicy Ignore): authz NoOpinion, admission
 * allow (cmd/cedar-webhook/main.go:116 allowOnError). */
int cg_batch_wait(cg_batch* b, int64_t timeout_ns);
/* Diagnostics of one batch's submit -> results interval (no reference counterpart; the bench's
 * split of it). cg_batch_set_profile(b, 1) before submit; after a successful wait,
 * cg_batch_profile fills up to n of, in ms: [0] string finalize, [1] host grouping, [2] the upload
 * call (pinned staging copy + enqueue of the H2D copies), [3] launch + D2H enqueue, then device
 * intervals from events on the batch's stream: [4] H2D copies, [5] the complete step, [6] the D2H
 * copy; [7] the wait call(s). */
int cg_batch_set_profile(cg_batch* b, int on);
int cg_batch_profile(cg_batch* b, double* ms, size_t n);
/* cedar.Decision for request i: *allow = 1 (Allow) / 0 (Deny); *tier = deciding tier index. */
int cg_batch_decision(cg_batch* b, uint32_t i, int* allow, uint32_t* tier);
/* json.Marshal(cedar.Diagnostic) (reasons_only=0) or json.Marshal(diagnostic.Reasons) (=1).
 * Writes at most cap bytes incl. NUL; *need = required size incl. NUL. */
int cg_batch_diagnostic(cg_batch* b, uint32_t i, int reasons_only, char* buf, size_t cap, size_t* need);
/* Determining-policy indices (image order) and error count for request i. */
int cg_batch_reasons(cg_batch* b, uint32_t i, uint32_t* idx, uint32_t cap, uint32_t* n, uint32_t* n_errors);
/* Re-runs the complete evaluation step of the resident batch `iters` times (the first pass, the
 * gather of unfinished requests and the on-device follow-up launches, exactly what
 * cg_batch_submit enqueues); device time via HIP events on the batch's stream. */
int cg_batch_time(cg_batch* b, uint32_t iters, float* ms_total);
/* The same with a HIP event at every phase boundary: ms_phase[7] receives each phase's device time
 * summed over the iterations (0 device grouping, 1 index scan or the whole one-kernel first pass,
 * 2 candidate pass, 3 follow-up gather, 4-6 the many-hit / long-list / structural follow-ups) and
 * ms_total the steps' total. */
#define CG_STEP_PHASES 7
int cg_batch_time_split(cg_batch* b, uint32_t iters, float* ms_phase, float* ms_total);
/* Requests of the batch whose result lists overflowed both the first pass and the on-device
 * follow-up and were re-run from the host by cg_batch_wait (diagnostic; valid once done). */
int cg_batch_reruns(cg_batch* b, uint32_t* n);
/* Requests finished by each on-device follow-up worklist: counts[0] many-hit (large-stage probe
 * kernel), [1] long reason / error lists (probe kernel), [2] structural comparisons (policy-stream
 * kernel). Valid once the batch is done. */
int cg_batch_followups(cg_batch* b, uint32_t* counts);
/* Device bytes of the batch (heap + results) and of its image. */
int cg_batch_bytes(cg_batch* b, uint64_t* batch_bytes, uint64_t* image_bytes, uint64_t* heap_bytes);
/* What the batch moves over PCIe once submitted: the one H2D upload (request heap, rows, strings,
 * grouping keys) and the one D2H result copy; and the ancestor-list words its requests carried and
 * how many of those an earlier request's interned copy served (image.h "ancestor lists"). */
int cg_batch_io(cg_batch* b, uint64_t* h2d_bytes, uint64_t* d2h_bytes, uint64_t* list_words, uint64_t* list_words_shared);

/* ---- authorization webhook path (SubjectAccessReview in, authorizer.Decision + reason out) ----
 * Appends SubjectAccessReview JSON objects (one or an array) as the reference's /v1/authorize
 * handler receives them (server.go:104). Applies GetAuthorizerAttributes (server.go:163-214), the
 * Authorize fast paths (authorizer.go:38-57: self-allow, `system:` bypass) and RecordToCedarResource
 * (authorizer.go:89-111); fast-path items are decided on the host and never reach the GPU.
 * Store readiness (authorizer.go:58-66) is the caller's check, done before this call. */
int cg_batch_add_sar_json(cg_batch* b, const char* json, size_t len);
/* Host-only: the (EntityMap, Request) the SAR path builds, as {"fast":d,"reason":r} for a fast-path
 * item or {"entities":[...],"request":{...}} (Cedar JSON) — for parity tests of the encoder. */
int cg_sar_to_cedar_json(const char* sar_json, size_t len, char* out, size_t cap, size_t* need);
/* Host-only consistency check of the SubjectAccessReview encoders: every element of the JSON
 * array `sars` goes through the direct path (views into the body, no trees) and the general path
 * (JSON tree -> Attributes -> entities -> encoder) for `image`; *n_direct counts the elements the
 * direct path took, *n_mismatch those whose encodings (or fast-path results) differ. */
int cg_encode_sar_check(const void* image, size_t len, const char* sars, size_t n, uint32_t* n_items,
                        uint32_t* n_direct, uint32_t* n_mismatch, int64_t* first_mismatch);
/* Host-only consistency check of the request encoder: every Cedar-JSON item of the array `items`
 * (cg_batch_add_json's format) is encoded twice for `image`, with the per-thread ancestor-record
 * cache and with the general hierarchy walk; *n_mismatch counts items whose encodings differ. */
int cg_encode_items_check(const void* image, size_t len, const char* items, size_t n, uint32_t* n_items,
                          uint32_t* n_mismatch, int64_t* first_mismatch);
/* Host-only consistency check of the bulk paths' JSON array splitter: `json` split into its top-level
 * elements by the serial scan and by the parallel one over `threads` regions; *n_elems = the element
 * count (-1: not an array), *same = 1 when both agree exactly. */
int cg_json_split_check(const char* json, size_t n, uint32_t threads, int64_t* n_elems, int* same);
/* authorizer.Decision for item i (0 Deny, 1 Allow, 2 NoOpinion) and the reason string the
 * reference returns (diagnosticToReason JSON, a fast-path literal, or ""). */
int cg_batch_authz(cg_batch* b, uint32_t i, int* decision, char* reason, size_t cap, size_t* need);

/* ---- admission webhook path (AdmissionReview in, allowed + status message out) ----
 * Appends AdmissionReview JSON objects ({"request": {...}}, a bare request object, or an array) as
 * the reference's /v1/admit handler receives them. Applies cedarHandler.Handle / review
 * (handler.go:43-153): the skipped namespaces (kube-system, cedar-k8s-authz-system), the principal
 * entities (entities/user.go), the resource entity flattened from the object / oldObject JSON
 * (UnstructuredToRecord + walkObject, entities/admission.go:123-369), the oldObject linkage, the
 * admission action entities and the request context. Store readiness (handler.go:49-57) is the
 * caller's check. The image must carry the trailing allow-all tier (cmd/cedar-webhook/main.go:111-116). */
int cg_batch_add_admission_json(cg_batch* b, const char* json, size_t len);
/* admission.Response for item i: *allowed; *code = 200, or 500 when the review failed
 * (admission.Errored; msg = the error text); msg = json.Marshal(diagnostics.Reasons) for a denial
 * with reasons (handler.go:62-66), else "". CG_E_RANGE: msg needs *need bytes. */
int cg_batch_admit(cg_batch* b, uint32_t i, int* allowed, int* code, char* msg, size_t cap, size_t* need);
/* Host-only: the (EntityMap, Request) the admission path builds, as Cedar JSON
 * {"entities":[...],"request":{...}}, or {"skip":true}, or {"error":"..."} — for encoder parity tests. */
int cg_admission_to_cedar_json(const char* review_json, size_t len, char* out, size_t cap, size_t* need);

/* ---- single-request drop-in: TieredPolicyStores.IsAuthorized(EntityMap, Request) ---- */
int cg_is_authorized_json(cg_ctx* ctx, const char* item_json, size_t len, int* allow, char* diag, size_t cap,
                          size_t* need);

/* ---- serving queue: concurrent blocking per-request calls, batched onto the device ----
 * Replaces the per-goroutine Authorize call of the webhook (authorizer.go:36-86; served by
 * server.go:104 /v1/authorize). Any number of threads call cg_queue_authorize_sar concurrently;
 * each call parses and converts its request on the calling thread, joins the open device batch
 * and blocks until that batch is evaluated. The batch is closed at max_batch requests or when
 * its first request has waited max_delay_us (0: as soon as the device is idle). */
typedef struct cg_queue cg_queue;
int cg_queue_create(cg_ctx* ctx, uint32_t max_batch, uint32_t max_delay_us, cg_queue** out);
/* The same queue over n_ctx contexts (one per GPU, §8(e)): one flusher builds the batches and deals
 * each to the least loaded GPU, whose submitter thread runs it. Requests are encoded against
 * ctxs[0]'s active image; a batch runs on the other context's image of that epoch (load it there
 * with cg_image_load_peer or the same blob), or on ctxs[0] while that context lacks the epoch. */
int cg_queue_create_multi(cg_ctx* const* ctxs, uint32_t n_ctx, uint32_t max_batch, uint32_t max_delay_us,
                          cg_queue** out);
/* Batches and requests the queue's k-th context (ctxs[k]) has run. */
int cg_queue_gpu_stats(cg_queue* q, uint32_t k, uint64_t* batches, uint64_t* requests);
/* Drains pending batches, then stops the flusher. No call may be in flight on q. */
void cg_queue_destroy(cg_queue* q);
/* Error text of the calling thread's last failed cg_queue_* call. */
const char* cg_queue_last_error(void);
/* authorizer.Decision (0 Deny, 1 Allow, 2 NoOpinion) and reason of one SubjectAccessReview, as
 * cg_batch_authz reports them. CG_E_RANGE: reason needs *need bytes (the decision is valid).
 * timeout_ns (< 0: none) bounds the whole call, counted from its entry: past it the call returns
 * CG_E_TIMEOUT (the request may still be evaluated; its result is dropped). On CG_E_TIMEOUT or
 * CG_E_DEVICE the caller answers NoOpinion (authorizer.go:80-84; the apiserver's failurePolicy). */
int cg_queue_authorize_sar(cg_queue* q, const char* sar_json, size_t len, int64_t timeout_ns, int* decision,
                           char* reason, size_t cap, size_t* need);
/* cg_queue_authorize_sar for n SubjectAccessReview bodies in one call: the entry point of a host-side
 * batcher (north_star's batching layer in internal/server: one goroutine collects the webhook
 * goroutines' requests and crosses into cgo once per group). The n requests are encoded on the
 * calling thread, join the open device batches together and the call blocks until all are
 * evaluated. decisions[k] as cg_queue_authorize_sar's; the reasons are written NUL-terminated side
 * by side into reasons[0..cap) with request k's at offsets[k] (any of reasons / offsets may be
 * NULL); *need receives the bytes they take, and CG_E_RANGE means reasons was too small (call
 * again with room). A deadline miss or device error fails the whole call (every request answers
 * NoOpinion). */
int cg_queue_authorize_sar_n(cg_queue* q, const char* const* sars, const size_t* lens, uint32_t n, int64_t timeout_ns,
                             int* decisions, char* reasons, size_t cap, size_t* offsets, size_t* need);
/* TieredPolicyStores.IsAuthorized for one Cedar-JSON item (cg_batch_add_json's format) through
 * the queue: *allow and, when diag or need is given, json.Marshal(cedar.Diagnostic). timeout_ns as
 * for cg_queue_authorize_sar; on CG_E_TIMEOUT / CG_E_DEVICE the admission caller allows. */
int cg_queue_is_authorized_json(cg_queue* q, const char* item_json, size_t len, int64_t timeout_ns, int* allow,
                                char* diag, size_t cap, size_t* need);
/* Counters: device batches run, requests through the device, fast-path requests, largest batch,
 * nanoseconds the flusher spent in submit + wait. Any pointer may be NULL. */
int cg_queue_stats(cg_queue* q, uint64_t* batches, uint64_t* requests, uint64_t* fast, uint64_t* max_batch,
                   uint64_t* device_ns);
/* Requests the queue dropped unevaluated because their callers' deadlines passed while they still
 * waited for a batch (the callers already returned CG_E_TIMEOUT and failed safe). */
int cg_queue_dropped(cg_queue* q, uint64_t* abandoned);

/* ---- metrics (the reference's cedar_authorizer_* collectors, metrics/metrics.go:27-65) ----
 * A snapshot of the queue's serving metrics for a Prometheus exporter on the host side:
 * - request_total{decision} and request_duration_seconds{decision}: every cg_queue_authorize_sar /
 *   cg_queue_is_authorized_json call, by outcome (Deny, Allow, NoOpinion, error; an admission call's
 *   allow counts as Allow, its deny as Deny), with its latency from entry to return; a call that
 *   returns CG_E_RANGE is not counted (its repeat with room for the reason is). The reference
 *   records only non-Deny decisions and errors (server.go:81-90): its exporter skips index 0.
 * - the batch-size and batch-latency (submit -> results published) histograms and the active
 *   image epoch that SURVEY §5 asks for beside them.
 * Latency buckets are "le" buckets over cg_metrics_latency_bounds (ns; 10 µs .. 10 s, a superset of
 * the reference's 0.25-10 s buckets, metrics.go:43), counted per bucket (not cumulative); the last
 * bucket is +Inf. Batch-size bucket k counts batches of size <= 2^k; the last one, the rest. */
#define CG_LAT_BOUNDS 21
#define CG_BATCH_BUCKETS 14
typedef struct cg_queue_metrics {
  uint64_t requests[4];                   /* by outcome: 0 Deny, 1 Allow, 2 NoOpinion, 3 error */
  uint64_t latency[4][CG_LAT_BOUNDS + 1]; /* per outcome, per latency bucket */
  uint64_t latency_sum_ns[4];
  uint64_t fast;                          /* answered on the host (fast path), included above */
  uint64_t batches;
  uint64_t batch_size[CG_BATCH_BUCKETS + 1];
  uint64_t batch_latency[CG_LAT_BOUNDS + 1];
  uint64_t batch_latency_sum_ns;
  uint64_t abandoned;                     /* cg_queue_dropped */
  uint64_t active_epoch;                  /* ctxs[0]'s active image (cg_image_active; 0: none) */
  uint64_t activations;                   /* cg_image_activate calls that switched ctxs[0]'s image */
} cg_queue_metrics;
/* The CG_LAT_BOUNDS bucket upper bounds in nanoseconds. */
const uint64_t* cg_metrics_latency_bounds(uint32_t* n);
/* Fills *out (size: sizeof(cg_queue_metrics), checked). Counters are read one by one (relaxed):
 * a snapshot taken while calls run may be a few calls apart between fields. */
int cg_queue_metrics_get(cg_queue* q, cg_queue_metrics* out, size_t size);
/* Bench support: `threads` threads issue `total` blocking cg_queue_authorize_sar calls cycling
 * over sars[0..n); wall seconds, per-call latency p50/p99/max (ns) and decision counts
 * counts[0..3) = (Deny, Allow, NoOpinion). */
int cg_queue_loadgen(cg_queue* q, const char* const* sars, const size_t* lens, uint32_t n, uint32_t threads,
                     uint64_t total, double* seconds, uint64_t* lat_p50, uint64_t* lat_p99, uint64_t* lat_max,
                     uint64_t* counts);
/* The same with each caller thread carrying per_call requests per cg_queue_authorize_sar_n call
 * (a request's latency is its call's). */
int cg_queue_loadgen_n(cg_queue* q, const char* const* sars, const size_t* lens, uint32_t n, uint32_t threads,
                       uint32_t per_call, uint64_t total, double* seconds, uint64_t* lat_p50, uint64_t* lat_p99,
                       uint64_t* lat_max, uint64_t* counts);

#ifdef __cplusplus
}
#endif
#endif /* CEDARGPU_H */
