"""Host-side mirror of the reference's policy stores and tier walk, driving the GPU C-ABI.

Reference interfaces mirrored (file:line in the reference):
  PolicyStore                      internal/server/store/store.go:9-15
  TieredPolicyStores.IsAuthorized  internal/server/store/store.go:25-42
  NewMemoryStore                   internal/server/store/memory.go:17-27   (IDs policy<i>)
  directory store                  internal/server/store/directory.go:41-82 (IDs <file>.policy<i>)
  CRD store                        internal/server/store/crd.go:45-118      (IDs <name><i>-<uid>)
  Verified Permissions store       internal/server/store/verified_permissions.go:58-100 (IDs <id>.<i>)
  StaticStore / allow-all          internal/server/store/memory.go:30-43, cmd/cedar-webhook/main.go:111-116
"""
from __future__ import annotations

import ctypes
import json
import threading
import time
import weakref
from typing import Iterable, List, Optional, Sequence, Tuple, Union

from ._lib import CG_E_RANGE, CompileError, DeadlineError, DeviceError, _err, lib

# an uninitialised bytes object of n bytes (filled by the library before it is returned)
_new_bytes = ctypes.pythonapi.PyBytes_FromStringAndSize
_new_bytes.restype = ctypes.py_object
_new_bytes.argtypes = [ctypes.c_void_p, ctypes.c_ssize_t]

FAULT_NONE, FAULT_DEVICE_ERROR, FAULT_STALL, FAULT_BAD_KIDX = 0, 1, 2, 3
DOC_SKIP_INVALID = 1
# Batch.route bits (include/cedargpu.h CG_ROUTE_*)
ROUTE_FU_BIG, ROUTE_FU_OVF, ROUTE_FU_GEN, ROUTE_FIRST_SLOT, ROUTE_RERUN, ROUTE_CLASS = 1, 2, 4, 8, 16, 32


def _timeout_ns(timeout: Optional[float]) -> int:
    return -1 if timeout is None else max(0, int(timeout * 1e9))


_P = ctypes.c_void_p


def _b(s) -> bytes:
    """UTF-8 bytes of a str; bytes (a request body as received) pass through without a copy."""
    return s if isinstance(s, (bytes, bytearray)) else s.encode("utf-8")


def device_count() -> int:
    n = ctypes.c_int(0)
    rc = lib.cg_device_count(ctypes.byref(n))
    return n.value if rc == 0 else 0


def device_synchronize(device: int = 0):
    rc = lib.cg_device_synchronize(device)
    if rc:
        raise DeviceError(rc, f"hipDeviceSynchronize failed on {device}")



LAT_BOUNDS, BATCH_BUCKETS = 21, 14  # include/cedargpu.h CG_LAT_BOUNDS, CG_BATCH_BUCKETS


class QueueMetrics(ctypes.Structure):
    """include/cedargpu.h cg_queue_metrics."""
    _fields_ = [
        ("requests", ctypes.c_uint64 * 4),
        ("latency", (ctypes.c_uint64 * (LAT_BOUNDS + 1)) * 4),
        ("latency_sum_ns", ctypes.c_uint64 * 4),
        ("fast", ctypes.c_uint64),
        ("batches", ctypes.c_uint64),
        ("batch_size", ctypes.c_uint64 * (BATCH_BUCKETS + 1)),
        ("batch_latency", ctypes.c_uint64 * (LAT_BOUNDS + 1)),
        ("batch_latency_sum_ns", ctypes.c_uint64),
        ("abandoned", ctypes.c_uint64),
        ("active_epoch", ctypes.c_uint64),
        ("activations", ctypes.c_uint64),
    ]

class PolicyStore:
    """A policy source. `documents()` yields (kind, args) fed to the compiler."""

    name = "PolicyStore"
    load_complete = True
    skip_invalid = False  # a document that does not parse fails the build (memory.go:17-22)

    def documents(self):
        raise NotImplementedError

    def initial_policy_load_complete(self) -> bool:
        return self.load_complete


class MemoryStore(PolicyStore):
    """store.NewMemoryStore(filename, document, loadComplete) — cedar.NewPolicySetFromBytes."""

    def __init__(self, filename: str, document: str, load_complete: bool = True):
        self.name = filename
        self.filename = filename
        self.document = document
        self.load_complete = load_complete

    def documents(self):
        yield ("doc", self.filename, self.document, "policy", "")


class DirectoryStore(PolicyStore):
    """Directory store snapshot: {file name: content} of the *.cedar files (directory.go:51-79)."""

    name = "FilePolicyStore"

    def __init__(self, files: dict):
        self.files = dict(files)

    skip_invalid = True  # a file that does not parse is logged and skipped (directory.go:69-73)

    def documents(self):
        for fname in sorted(self.files):  # os.ReadDir returns entries sorted by filename
            if not fname.endswith(".cedar"):
                continue
            yield ("doc", fname, self.files[fname], f"{fname}.policy", "")


class CRDStore(PolicyStore):
    """Policy CRD snapshot: list of (metadata.name, metadata.uid, spec.content) (crd.go:45-118)."""

    name = "CRDPolicyStore"
    skip_invalid = True  # a CRD that does not parse contributes nothing (crd.go:51-55, 83-95)

    def __init__(self, policies: Sequence[Tuple[str, str, str]]):
        self.policies = list(policies)

    def documents(self):
        for name, uid, content in self.policies:
            yield ("doc", name, content, name, f"-{uid}")


class AVPStore(PolicyStore):
    """Amazon Verified Permissions snapshot: list of (policyId, statement) (verified_permissions.go:58-100)."""

    name = "VerifiedPermissionsPolicyStore"
    skip_invalid = True  # a statement that does not parse is skipped (verified_permissions.go:89-93)

    def __init__(self, policies: Sequence[Tuple[str, str]]):
        self.policies = list(policies)

    def documents(self):
        for pid, stmt in self.policies:
            yield ("doc", pid, stmt, f"{pid}.", "")


class StaticStore(PolicyStore):
    """StaticStore built from AST policies: explicit IDs, zero Position (admit_all_policy.go:10-19)."""

    name = "StaticStore"

    def __init__(self, policies: Sequence[Tuple[str, str]]):
        self.policies = list(policies)

    def documents(self):
        for pid, text in self.policies:
            yield ("policy", pid, "", text, True)


ALLOW_ALL_ADMISSION = StaticStore([(
    "allow-all-admission",
    'permit (principal, action in [k8s::admission::Action::"create", k8s::admission::Action::"update", '
    'k8s::admission::Action::"delete", k8s::admission::Action::"connect"], resource);')])


class Compiler:
    """A policy compiler that keeps parsed and lowered documents across builds (cg_compiler_*): the
    incremental rebuild a store change triggers parses and lowers only the new or changed
    documents (`incremental=False`: every build a full one, byte-identical to a fresh compiler's)."""

    def __init__(self, incremental: bool = True):
        self._h = _P()
        if lib.cg_compiler_create(ctypes.byref(self._h)):
            raise CompileError(-1, "compiler create failed")
        if not incremental:
            lib.cg_compiler_set_incremental(self._h, 0)

    def last_build(self) -> dict:
        """{"incremental", "lowered", "reused", "why_full"} of the last build (cg_compiler_last_build)."""
        inc, lo, re = ctypes.c_int(), ctypes.c_uint64(), ctypes.c_uint64()
        why = ctypes.c_char_p()
        rc = lib.cg_compiler_last_build(self._h, ctypes.byref(inc), ctypes.byref(lo), ctypes.byref(re), ctypes.byref(why))
        if rc:
            raise _err(rc, "last_build failed")
        return {"incremental": bool(inc.value), "lowered": lo.value, "reused": re.value,
                "why_full": (why.value or b"").decode()}

    def close(self):
        if self._h:
            lib.cg_compiler_destroy(self._h)
            self._h = _P()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def build(self, stores: Sequence[PolicyStore], epoch: int = 1, entities: Optional[list] = None) -> bytes:
        """Compiles the tiers. `entities`: the image's static entities (Cedar JSON entity list, e.g.
        a group hierarchy), merged into every request's EntityMap (cg_compiler_set_entities)."""
        c = self._h
        t0 = time.perf_counter()
        lib.cg_compiler_clear(c)
        eb = _b(json.dumps(entities)) if entities else b""
        rc = lib.cg_compiler_set_entities(c, eb, len(eb))
        if rc:
            raise _err(rc, lib.cg_compiler_last_error(c).decode())
        for st in stores:
            lib.cg_compiler_add_tier(c)
            for d in st.documents():
                if d[0] == "doc":
                    _, fname, text, pre, suf = d
                    tb = _b(text)
                    rc = lib.cg_compiler_add_document_ex(c, _b(fname), tb, len(tb), _b(pre), _b(suf),
                                                         DOC_SKIP_INVALID if st.skip_invalid else 0)
                else:
                    _, pid, fname, text, zero = d
                    tb = _b(text)
                    rc = lib.cg_compiler_add_policy(c, _b(pid), _b(fname), tb, len(tb), 1 if zero else 0)
                if rc:
                    raise _err(rc, lib.cg_compiler_last_error(c).decode())
        # the blob is serialized straight into a new bytes object (cg_compiler_build_sized, then
        # cg_compiler_write_image into its storage before anything else can see it): no second
        # copy of a 100 MB image
        n = ctypes.c_size_t(0)
        t1 = time.perf_counter()
        rc = lib.cg_compiler_build_sized(c, epoch, ctypes.byref(n))
        if rc:
            raise _err(rc, lib.cg_compiler_last_error(c).decode())
        t2 = time.perf_counter()
        blob = _new_bytes(None, n.value)
        rc = lib.cg_compiler_write_image(c, ctypes.cast(ctypes.c_char_p(blob), ctypes.c_void_p), n.value)
        if rc:
            raise _err(rc, lib.cg_compiler_last_error(c).decode())
        # seconds spent handing over the documents, compiling, and writing the blob
        self.last_times = {"documents": t1 - t0, "compile": t2 - t1, "blob": time.perf_counter() - t2}
        return blob

    def doc_errors(self) -> List[dict]:
        """[{"filename", "error"}] of the documents the last build left out (skip_invalid stores)."""
        need = ctypes.c_size_t(0)
        lib.cg_compiler_doc_errors(self._h, None, 0, ctypes.byref(need))
        buf = ctypes.create_string_buffer(max(need.value, 3))
        rc = lib.cg_compiler_doc_errors(self._h, buf, len(buf), ctypes.byref(need))
        if rc:
            raise _err(rc, "doc_errors failed")
        return json.loads(buf.value.decode("utf-8"))

    def cache_stats(self) -> dict:
        v = [ctypes.c_uint64() for _ in range(3)]
        lib.cg_compiler_cache_stats(self._h, *[ctypes.byref(x) for x in v])
        return dict(zip(("hits", "misses", "entries"), (x.value for x in v)))


def build_image(stores: Sequence[PolicyStore], epoch: int = 1, entities: Optional[list] = None) -> bytes:
    """Compiles the tiers (one per store), and the static entities, into an image blob. Host only."""
    c = Compiler()
    try:
        return c.build(stores, epoch, entities)
    finally:
        c.close()


def image_stats(image: bytes) -> dict:
    """Shape of a compiled image: policies, tiers, atom-lowered policies, hot attributes, ..."""
    u = [ctypes.c_uint32() for _ in range(6)]
    ep = ctypes.c_uint64()
    if lib.cg_image_info(image, len(image), ctypes.byref(u[0]), ctypes.byref(u[1]), ctypes.byref(ep)):
        raise ValueError("not a compiled policy image")
    lib.cg_image_stats(image, len(image), *(ctypes.byref(x) for x in u[2:]))
    ix = ctypes.c_int(0)
    lib.cg_image_indexed(image, len(image), ctypes.byref(ix))
    lw, lr = ctypes.c_uint32(), ctypes.c_uint32()
    lib.cg_image_like_slots(image, len(image), ctypes.byref(lw), ctypes.byref(lr))
    return {"policies": u[0].value, "tiers": u[1].value, "epoch": ep.value, "atomic": u[2].value,
            "hot": u[3].value, "actions": u[4].value, "stream_words": u[5].value, "indexed": bool(ix.value),
            "row_like_slots": bin(lw.value).count("1"), "like_read_mask": lr.value}


def _buf(b: bytes):
    return ctypes.cast(ctypes.c_char_p(b), ctypes.c_void_p)  # the bytes' own buffer (read only)


def image_delta(base: bytes, new: bytes) -> bytes:
    """cg_image_delta: the delta image that turns blob `base` into blob `new` (include/cedargpu.h)."""
    out, n = _P(), ctypes.c_size_t(0)
    rc = lib.cg_image_delta(_buf(base), len(base), _buf(new), len(new), ctypes.byref(out), ctypes.byref(n))
    if rc:
        raise _err(rc, "image delta failed")
    try:
        return ctypes.string_at(out, n.value)
    finally:
        lib.cg_free(out)


def image_patch(base: bytes, delta: bytes) -> bytes:
    """cg_image_patch: base + delta on the host (raises on a malformed delta or another base)."""
    out, n = _P(), ctypes.c_size_t(0)
    rc = lib.cg_image_patch(_buf(base), len(base), _buf(delta), len(delta), ctypes.byref(out), ctypes.byref(n))
    if rc:
        raise _err(rc, "delta does not apply to this base")
    try:
        return ctypes.string_at(out, n.value)
    finally:
        lib.cg_free(out)


def delta_info(delta: bytes) -> dict:
    v = [ctypes.c_uint64() for _ in range(4)]
    if lib.cg_delta_info(_buf(delta), len(delta), *(ctypes.byref(x) for x in v)):
        raise ValueError("not a delta image")
    return dict(zip(("base_len", "new_len", "ops", "literal_bytes"), (x.value for x in v)))


def index_stats(image: bytes) -> dict:
    """Scope-index shape of a compiled image (cg_image_index_stats): list-keyed hot slots, key
    combos, index entries, scope-bitset contexts."""
    u = [ctypes.c_uint32() for _ in range(6)]
    if lib.cg_image_index_stats(image, len(image), *(ctypes.byref(x) for x in u)):
        raise ValueError("not a compiled policy image")
    return dict(zip(("cslot_mask", "pslot_mask", "combo_mask", "entries", "contexts", "sbits_words"),
                    (x.value for x in u)))


def atomic_policies(image: bytes) -> List[bool]:
    """Per policy (image order): lowered to predicate atoms (True) or bytecode."""
    n = image_stats(image)["policies"]
    out = []
    for i in range(n):
        a = ctypes.c_int(0)
        lib.cg_image_policy_atomic(image, len(image), i, ctypes.byref(a))
        out.append(bool(a.value))
    return out


class Context:
    """One GPU: loaded images (by epoch) and the active one."""

    def __init__(self, device: int = 0):
        self.device = device
        self._h = _P()
        self._batches = weakref.WeakSet()  # open batches: a batch never outlives its context
        rc = lib.cg_ctx_create(device, ctypes.byref(self._h))
        if rc:
            raise DeviceError(rc, f"no usable GPU {device}: {lib.cg_last_error(None).decode()}")

    def close(self):
        if self._h:
            # (cg_batch_destroy needs its context: a batch still referenced somewhere, e.g. by a
            # failed test's traceback, is closed here rather than later against a freed context)
            for b in list(self._batches):
                b.close()
            lib.cg_ctx_destroy(self._h)
            self._h = _P()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def last_error(self) -> str:
        return lib.cg_last_error(self._h).decode()

    def load(self, image: bytes, epoch: int, activate: bool = True):
        buf = ctypes.cast(ctypes.c_char_p(image), ctypes.c_void_p)  # the bytes' own buffer (cg_image_load copies)
        rc = lib.cg_image_load(self._h, buf, len(image), epoch)
        if rc:
            raise _err(rc, self.last_error())
        if activate:
            rc = lib.cg_image_activate(self._h, epoch)
            if rc:
                raise _err(rc, self.last_error())

    def load_peer(self, src: "Context", epoch: int, activate: bool = True):
        """cg_image_load_peer: `src`'s image for `epoch`, host tables shared, device copy GPU to GPU."""
        rc = lib.cg_image_load_peer(self._h, src._h, epoch)
        if rc:
            raise _err(rc, self.last_error())
        if activate:
            self.activate(epoch)

    def load_delta(self, base_epoch: int, delta: bytes, epoch: int, activate: bool = True):
        """cg_image_load_delta: the image `delta` makes of this context's `base_epoch` image, built
        on the GPU from the base's device copy, loaded as `epoch`."""
        rc = lib.cg_image_load_delta(self._h, base_epoch, _buf(delta), len(delta), epoch)
        if rc:
            raise _err(rc, self.last_error())
        if activate:
            self.activate(epoch)

    def activate(self, epoch: int):
        rc = lib.cg_image_activate(self._h, epoch)
        if rc:
            raise _err(rc, self.last_error())

    def batch(self) -> "Batch":
        return Batch(self)

    def inject_fault(self, kind: int, arg: int = 0):
        """Gameday fault injection (cg_ctx_inject_fault): FAULT_DEVICE_ERROR fails the next `arg`
        submits, FAULT_STALL delays every batch by `arg` microseconds on the device, FAULT_BAD_KIDX
        makes the next `arg` batches carry key-entity indices of another image (they fail)."""
        rc = lib.cg_ctx_inject_fault(self._h, kind, arg)
        if rc:
            raise _err(rc, "inject_fault failed")


def pinned_stats() -> dict:
    """cg_pinned_stats: the encoder's process-wide pinned pool (bytes held, idle blocks) and the
    number of batches closed in flight that kept their arrays until their stream drained."""
    held, idle, kept = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
    lib.cg_pinned_stats(ctypes.byref(held), ctypes.byref(idle), ctypes.byref(kept))
    return {"held_bytes": held.value, "idle_blocks": idle.value, "kept_batches": kept.value}


class Batch:
    def __init__(self, ctx: Context):
        self.ctx = ctx
        self._h = _P()
        rc = lib.cg_batch_create(ctx._h, ctypes.byref(self._h))
        if rc:
            raise _err(rc, ctx.last_error())
        ctx._batches.add(self)

    def close(self):
        if self._h:
            lib.cg_batch_destroy(self._h)
            self._h = _P()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def add_json(self, payload: str):
        b = _b(payload)
        rc = lib.cg_batch_add_json(self._h, b, len(b))
        if rc:
            raise _err(rc, "batch add failed")

    def add(self, entities: list, request: dict):
        self.add_json(json.dumps({"entities": entities, "request": request}))

    def add_sar_json(self, payload):
        """SubjectAccessReview JSON (object or array; str, or bytes as received) -> entities via the
        C++ model (sar.cpp)."""
        b = _b(payload)
        rc = lib.cg_batch_add_sar_json(self._h, b, len(b))
        if rc:
            raise _err(rc, "SubjectAccessReview encode failed")

    def add_admission_json(self, payload):
        """AdmissionReview JSON (object or array) -> entities via the C++ model (admission.cpp)."""
        b = _b(payload)
        rc = lib.cg_batch_add_admission_json(self._h, b, len(b))
        if rc:
            raise _err(rc, "AdmissionReview encode failed")

    def admit(self, i: int) -> Tuple[bool, int, str]:
        """(allowed, HTTP status code, message) of admission.Response — handler.go:43-80."""
        allowed, code = ctypes.c_int(), ctypes.c_int()
        need = ctypes.c_size_t(0)
        buf = ctypes.create_string_buffer(512)
        rc = lib.cg_batch_admit(self._h, i, ctypes.byref(allowed), ctypes.byref(code), buf, 512, ctypes.byref(need))
        if rc == CG_E_RANGE and need.value > 512:
            buf = ctypes.create_string_buffer(need.value)
            rc = lib.cg_batch_admit(self._h, i, ctypes.byref(allowed), ctypes.byref(code), buf, need.value,
                                    ctypes.byref(need))
        if rc:
            raise _err(rc, "admission result failed")
        return bool(allowed.value), code.value, buf.value.decode("utf-8")

    def authz(self, i: int) -> Tuple[int, str]:
        """(authorizer.Decision: 0 Deny / 1 Allow / 2 NoOpinion, reason) — authorizer.go:36-85."""
        dec = ctypes.c_int()
        need = ctypes.c_size_t(0)
        buf = ctypes.create_string_buffer(512)
        rc = lib.cg_batch_authz(self._h, i, ctypes.byref(dec), buf, 512, ctypes.byref(need))
        if rc == CG_E_RANGE and need.value > 512:
            buf = ctypes.create_string_buffer(need.value)
            rc = lib.cg_batch_authz(self._h, i, ctypes.byref(dec), buf, need.value, ctypes.byref(need))
        if rc:
            raise _err(rc, "authz result failed")
        return dec.value, buf.value.decode("utf-8")

    def __len__(self):
        return lib.cg_batch_size(self._h)

    def submit(self):
        rc = lib.cg_batch_submit(self._h)
        if rc:
            raise _err(rc, "batch submit failed")

    def wait(self, timeout: Optional[float] = None):
        """cg_batch_wait; raises DeadlineError past `timeout` seconds (the batch stays in flight)."""
        rc = lib.cg_batch_wait(self._h, _timeout_ns(timeout))
        if rc:
            raise _err(rc, "batch wait failed")

    def decision(self, i: int) -> Tuple[bool, int]:
        allow = ctypes.c_int()
        tier = ctypes.c_uint32()
        rc = lib.cg_batch_decision(self._h, i, ctypes.byref(allow), ctypes.byref(tier))
        if rc:
            raise _err(rc, "decision failed")
        return bool(allow.value), tier.value

    def diagnostic(self, i: int, reasons_only: bool = False) -> str:
        need = ctypes.c_size_t(0)
        buf = ctypes.create_string_buffer(512)
        rc = lib.cg_batch_diagnostic(self._h, i, 1 if reasons_only else 0, buf, 512, ctypes.byref(need))
        if rc == CG_E_RANGE and need.value > 512:
            buf = ctypes.create_string_buffer(need.value)
            rc = lib.cg_batch_diagnostic(self._h, i, 1 if reasons_only else 0, buf, need.value, ctypes.byref(need))
        if rc:
            raise _err(rc, "diagnostic failed")
        return buf.value.decode("utf-8")

    def reasons(self, i: int) -> Tuple[List[int], int]:
        n = ctypes.c_uint32()
        ne = ctypes.c_uint32()
        lib.cg_batch_reasons(self._h, i, None, 0, ctypes.byref(n), ctypes.byref(ne))
        arr = (ctypes.c_uint32 * max(n.value, 1))()
        rc = lib.cg_batch_reasons(self._h, i, arr, n.value, ctypes.byref(n), ctypes.byref(ne))
        if rc:
            raise _err(rc, "reasons failed")
        return list(arr[:n.value]), ne.value

    def route(self, i: int) -> int:
        """How request i was finished: CG_ROUTE_* bits (ROUTE_* below; 0: the first pass alone)."""
        return self.route_words(i)[0]

    def route_words(self, i: int) -> Tuple[int, int]:
        """(route bits, reason words the device wrote for request i's deciding list)."""
        r, w = ctypes.c_uint32(0), ctypes.c_uint32(0)
        rc = lib.cg_batch_route(self._h, i, ctypes.byref(r), ctypes.byref(w))
        if rc:
            raise _err(rc, "route failed")
        return r.value, w.value

    def reruns(self) -> int:
        """Requests whose result lists overflowed the first pass and were re-run (cg_batch_reruns)."""
        n = ctypes.c_uint32()
        rc = lib.cg_batch_reruns(self._h, ctypes.byref(n))
        if rc:
            raise _err(rc, "reruns failed")
        return n.value

    def followups(self) -> dict:
        """Requests finished by each on-device follow-up worklist (cg_batch_followups)."""
        c = (ctypes.c_uint32 * 3)()
        rc = lib.cg_batch_followups(self._h, c)
        if rc:
            raise _err(rc, "followups failed")
        return {"big": c[0], "long_lists": c[1], "structural": c[2]}

    def time(self, iters: int) -> float:
        ms = ctypes.c_float()
        rc = lib.cg_batch_time(self._h, iters, ctypes.byref(ms))
        if rc:
            raise _err(rc, "timing failed")
        return ms.value

    PHASES = ("group", "scan", "candidates", "gather", "fu_big", "fu_long_lists", "fu_structural")

    def time_split(self, iters: int):
        """(per-phase device ms summed over `iters` steps, total ms): HIP events at each phase boundary
        of the complete step (cg_batch_time_split)."""
        ph = (ctypes.c_float * len(self.PHASES))()
        tot = ctypes.c_float()
        rc = lib.cg_batch_time_split(self._h, iters, ph, ctypes.byref(tot))
        if rc:
            raise _err(rc, "timing failed")
        return dict(zip(self.PHASES, list(ph))), tot.value

    def bytes(self):
        a, b, c = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        lib.cg_batch_bytes(self._h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c))
        return a.value, b.value, c.value

    def set_profile(self, on: bool = True):
        """cg_batch_set_profile: time this batch's submit -> results phases (before submit)."""
        rc = lib.cg_batch_set_profile(self._h, 1 if on else 0)
        if rc:
            raise _err(rc, "set_profile failed")

    def profile(self) -> dict:
        """cg_batch_profile: the submit -> results split of a profiled batch (ms)."""
        v = (ctypes.c_double * 8)()
        rc = lib.cg_batch_profile(self._h, v, 8)
        if rc:
            raise _err(rc, "profile failed")
        keys = ("host_finalize", "host_group", "host_upload_call", "host_launch", "dev_h2d", "dev_step", "dev_d2h", "host_wait")
        return dict(zip(keys, list(v)))

    def io(self) -> dict:
        """PCIe bytes of the submitted batch (one H2D upload, one D2H result copy) and its ancestor-
        list words, total and served by an interned copy (cg_batch_io)."""
        v = [ctypes.c_uint64() for _ in range(4)]
        rc = lib.cg_batch_io(self._h, *(ctypes.byref(x) for x in v))
        if rc:
            raise _err(rc, "batch io failed")
        return dict(zip(("h2d_bytes", "d2h_bytes", "list_words", "list_words_shared"), (x.value for x in v)))


class Queue:
    """Serving queue (cg_queue_*): blocking per-request calls from many threads, batched onto the
    device. `authorize` is the webhook's Authorize (authorizer.go:36-86) for one
    SubjectAccessReview; `is_authorized` is TieredPolicyStores.IsAuthorized for one Cedar-JSON item.
    ctypes releases the GIL for the duration of each call, so Python threads batch together."""

    def __init__(self, ctx: Union[Context, Sequence[Context]], max_batch: int = 4096, max_delay_us: int = 0):
        """`ctx`: one context, or one per GPU (cg_queue_create_multi: batches dealt to the least
        loaded GPU; requests encode against the first context's active image)."""
        ctxs = list(ctx) if isinstance(ctx, (list, tuple)) else [ctx]
        self.ctx = ctxs[0]
        self.ctxs = ctxs
        self._h = _P()
        arr = (_P * len(ctxs))(*[c._h for c in ctxs])
        rc = lib.cg_queue_create_multi(arr, len(ctxs), max_batch, max_delay_us, ctypes.byref(self._h))
        if rc:
            raise _err(rc, "queue create failed")

    def gpu_stats(self) -> List[dict]:
        """Per context: batches and requests it ran."""
        out = []
        for k in range(len(self.ctxs)):
            b, r = ctypes.c_uint64(), ctypes.c_uint64()
            lib.cg_queue_gpu_stats(self._h, k, ctypes.byref(b), ctypes.byref(r))
            out.append({"batches": b.value, "requests": r.value})
        return out

    def close(self):
        if self._h:
            lib.cg_queue_destroy(self._h)
            self._h = _P()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _call(self, fn, payload: str, timeout: Optional[float]) -> Tuple[int, str]:
        b = _b(payload)
        out = ctypes.c_int()
        need = ctypes.c_size_t(0)
        buf = ctypes.create_string_buffer(1024)
        rc = fn(self._h, b, len(b), _timeout_ns(timeout), ctypes.byref(out), buf, 1024, ctypes.byref(need))
        if rc == CG_E_RANGE and need.value > 1024:
            buf = ctypes.create_string_buffer(need.value)
            rc = fn(self._h, b, len(b), _timeout_ns(timeout), ctypes.byref(out), buf, need.value, ctypes.byref(need))
        if rc:
            raise _err(rc, lib.cg_queue_last_error().decode())
        return out.value, buf.value.decode("utf-8")

    def authorize(self, sar: Union[dict, str], timeout: Optional[float] = None) -> Tuple[int, str]:
        """(authorizer.Decision: 0 Deny / 1 Allow / 2 NoOpinion, reason). Raises DeadlineError past
        `timeout` seconds and DeviceError on a device failure (see `authorize_failsafe`)."""
        return self._call(lib.cg_queue_authorize_sar, sar if isinstance(sar, str) else json.dumps(sar), timeout)

    def authorize_failsafe(self, sar: Union[dict, str], timeout: Optional[float] = None) -> Tuple[int, str]:
        """authorize() with the webhook's fail-safe: a deadline or device failure answers NoOpinion
        with no reason, as the apiserver's failurePolicy NoOpinion would on a webhook timeout
        (mount/authorization-config.yaml:11,16) and as Authorize does without an opinion
        (authorizer.go:80-84)."""
        try:
            return self.authorize(sar, timeout)
        except (DeadlineError, DeviceError):
            return Authorizer.NO_OPINION, ""

    def is_authorized(self, entities: list, request: dict, timeout: Optional[float] = None) -> Tuple[bool, str]:
        """(allow, json.Marshal(cedar.Diagnostic))."""
        allow, diag = self._call(lib.cg_queue_is_authorized_json, json.dumps({"entities": entities, "request": request}),
                                 timeout)
        return bool(allow), diag

    def stats(self) -> dict:
        v = [ctypes.c_uint64() for _ in range(5)]
        rc = lib.cg_queue_stats(self._h, *[ctypes.byref(x) for x in v])
        if rc:
            raise _err(rc, "queue stats failed")
        out = dict(zip(("batches", "requests", "fast", "max_batch", "device_ns"), (x.value for x in v)))
        d = ctypes.c_uint64()
        if lib.cg_queue_dropped(self._h, ctypes.byref(d)) == 0:
            out["dropped"] = d.value
        return out

    def metrics(self) -> dict:
        """cg_queue_metrics_get: request_total / request_duration by outcome (Deny, Allow, NoOpinion,
        error), batch-size and batch-latency histograms, the active epoch (metrics.go:27-65)."""
        m = QueueMetrics()
        rc = lib.cg_queue_metrics_get(self._h, ctypes.byref(m), ctypes.sizeof(m))
        if rc:
            raise _err(rc, "queue metrics failed")
        n = ctypes.c_uint32()
        bp = lib.cg_metrics_latency_bounds(ctypes.byref(n))
        outcomes = ("deny", "allow", "no_opinion", "error")
        return {
            "latency_bounds_ns": [bp[i] for i in range(n.value)],
            "requests": {o: m.requests[i] for i, o in enumerate(outcomes)},
            "latency": {o: list(m.latency[i]) for i, o in enumerate(outcomes)},
            "latency_sum_ns": {o: m.latency_sum_ns[i] for i, o in enumerate(outcomes)},
            "fast": m.fast, "batches": m.batches,
            "batch_size": list(m.batch_size), "batch_latency": list(m.batch_latency),
            "batch_latency_sum_ns": m.batch_latency_sum_ns,
            "abandoned": m.abandoned, "active_epoch": m.active_epoch, "activations": m.activations,
        }

    def authorize_many(self, sars: Sequence[Union[dict, str]], timeout: Optional[float] = None) -> List[Tuple[int, str]]:
        """cg_queue_authorize_sar_n: several SubjectAccessReviews in one blocking call (a host-side
        batcher's entry point); [(decision, reason)] in order."""
        enc = [_b(s if isinstance(s, str) else json.dumps(s)) for s in sars]
        n = len(enc)
        arr = (ctypes.c_char_p * max(n, 1))(*enc)
        lens = (ctypes.c_size_t * max(n, 1))(*[len(e) for e in enc])
        dec = (ctypes.c_int * max(n, 1))()
        offs = (ctypes.c_size_t * max(n, 1))()
        need = ctypes.c_size_t(0)
        buf = ctypes.create_string_buffer(max(4096, 512 * n))
        for _ in range(2):
            rc = lib.cg_queue_authorize_sar_n(self._h, arr, lens, n, _timeout_ns(timeout), dec, buf, len(buf), offs,
                                              ctypes.byref(need))
            if rc != CG_E_RANGE:
                break
            buf = ctypes.create_string_buffer(need.value)
        if rc:
            raise _err(rc, lib.cg_queue_last_error().decode())
        raw = buf.raw
        return [(dec[k], raw[offs[k]:raw.index(b"\0", offs[k])].decode("utf-8")) for k in range(n)]

    def loadgen(self, sars_json: Sequence[str], threads: int, total: int, per_call: int = 1) -> dict:
        """Bench support: `threads` native threads issue `total` blocking authorize calls
        (`per_call` > 1: cg_queue_authorize_sar_n calls of that many requests each)."""
        enc = [_b(s) for s in sars_json]
        arr = (ctypes.c_char_p * len(enc))(*enc)
        lens = (ctypes.c_size_t * len(enc))(*[len(e) for e in enc])
        secs = ctypes.c_double()
        p50, p99, mx = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        counts = (ctypes.c_uint64 * 3)()
        rc = lib.cg_queue_loadgen_n(self._h, arr, lens, len(enc), threads, per_call, total, ctypes.byref(secs),
                                    ctypes.byref(p50), ctypes.byref(p99), ctypes.byref(mx), counts)
        if rc:
            raise _err(rc, lib.cg_queue_last_error().decode())
        return {"seconds": secs.value, "p50_us": p50.value / 1e3, "p99_us": p99.value / 1e3, "max_us": mx.value / 1e3,
                "deny": counts[0], "allow": counts[1], "no_opinion": counts[2]}


class TieredPolicyStores:
    """store.TieredPolicyStores over GPU-compiled tiers (store.go:20-42).

    `is_authorized(entities, request)` returns (decision: bool, diagnostic_json: str) exactly as
    the reference's TieredPolicyStores.IsAuthorized + json.Marshal(diagnostic) would.
    """

    _epoch_lock = threading.Lock()
    _next_epoch = 1

    def __init__(self, stores: Sequence[PolicyStore], device: int = 0, ctx: Optional[Context] = None,
                 entities: Optional[list] = None):
        self.stores = list(stores)
        self.entities = entities  # static entities merged into every EntityMap (a group hierarchy)
        self.ctx = ctx or Context(device)
        self.reload()

    def reload(self):
        """Recompiles every store and atomically swaps the active image (hot reload)."""
        with TieredPolicyStores._epoch_lock:
            epoch = TieredPolicyStores._next_epoch
            TieredPolicyStores._next_epoch += 1
        self.image = build_image(self.stores, epoch, self.entities)
        self.ctx.load(self.image, epoch, activate=True)
        self.epoch = epoch

    def ready(self) -> bool:
        return all(s.initial_policy_load_complete() for s in self.stores)

    def is_authorized_batch(self, items: Iterable[Tuple[list, dict]]) -> List[Tuple[bool, str]]:
        b = self.ctx.batch()
        payload = json.dumps([{"entities": e, "request": r} for e, r in items])
        b.add_json(payload)
        b.submit()
        b.wait()
        out = []
        for i in range(len(b)):
            ok, _ = b.decision(i)
            out.append((ok, b.diagnostic(i)))
        b.close()
        return out

    def is_authorized(self, entities: list, request: dict) -> Tuple[bool, str]:
        return self.is_authorized_batch([(entities, request)])[0]


class Authorizer:
    """cedarWebhookAuthorizer over GPU tiers (authorizer.go:21-85). `authorize_batch` takes
    SubjectAccessReview dicts and returns [(authorizer.Decision, reason)]."""

    DENY, ALLOW, NO_OPINION = 0, 1, 2

    def __init__(self, stores: Sequence[PolicyStore], device: int = 0, ctx: Optional[Context] = None,
                 timeout: Optional[float] = None, entities: Optional[list] = None):
        self.tiers = TieredPolicyStores(stores, device=device, ctx=ctx, entities=entities)
        self._loaded = False
        self.timeout = timeout  # per batch, seconds (the apiserver allows 3 s: authorization-config.yaml:11)

    def authorize_batch(self, sars: Sequence[dict]) -> List[Tuple[int, str]]:
        """Fail-safe: a device failure or a missed deadline answers NoOpinion for every request
        that needed the device (fast-path answers stand), as the apiserver's failurePolicy would."""
        if not self._loaded:  # authorizer.go:58-66 (checked after the fast paths there; see below)
            if not self.tiers.ready():
                return [_fast_or_noopinion(s) for s in sars]
            self._loaded = True
        b = self.tiers.ctx.batch()
        try:
            b.add_sar_json(json.dumps(list(sars)))
            try:
                b.submit()
                b.wait(self.timeout)
            except (DeviceError, DeadlineError):
                return [_fast_or_noopinion(s) for s in sars]
            return [b.authz(i) for i in range(len(b))]
        finally:
            b.close()

    def authorize(self, sar: dict) -> Tuple[int, str]:
        return self.authorize_batch([sar])[0]


class AdmissionHandler:
    """cedarHandler over GPU tiers (handler.go:43-167). The last store should be
    `ALLOW_ALL_ADMISSION` (main.go:111-116). `handle_batch` takes AdmissionReview dicts and returns
    [(allowed, HTTP status code, message)]."""

    def __init__(self, stores: Sequence[PolicyStore], device: int = 0, ctx: Optional[Context] = None,
                 timeout: Optional[float] = None, entities: Optional[list] = None):
        self.tiers = TieredPolicyStores(stores, device=device, ctx=ctx, entities=entities)
        self.timeout = timeout  # per batch, seconds (the webhook allows 30 s: admission-webhook.yaml:26)

    def handle_batch(self, reviews: Sequence[dict]) -> List[Tuple[bool, int, str]]:
        """Fail-safe: a device failure or a missed deadline allows every review (allowOnError,
        cmd/cedar-webhook/main.go:116; failurePolicy Ignore, manifests/admission-webhook.yaml:11)."""
        if not self.tiers.ready():  # handler.go:49-57: allow until every store has loaded
            return [(True, 200, "") for _ in reviews]
        b = self.tiers.ctx.batch()
        try:
            b.add_admission_json(json.dumps(list(reviews)))
            try:
                b.submit()
                b.wait(self.timeout)
            except (DeviceError, DeadlineError):
                return [(True, 200, "") for _ in reviews]
            return [b.admit(i) for i in range(len(b))]
        finally:
            b.close()

    def handle(self, review: dict) -> Tuple[bool, int, str]:
        return self.handle_batch([review])[0]


def admission_to_cedar_json(review: dict) -> dict:
    """Host-only: the (EntityMap, Request) the admission path builds (cg_admission_to_cedar_json)."""
    b = _b(json.dumps(review))
    need = ctypes.c_size_t(0)
    buf = ctypes.create_string_buffer(1 << 16)
    rc = lib.cg_admission_to_cedar_json(b, len(b), buf, 1 << 16, ctypes.byref(need))
    if rc == CG_E_RANGE and need.value > (1 << 16):
        buf = ctypes.create_string_buffer(need.value)
        rc = lib.cg_admission_to_cedar_json(b, len(b), buf, need.value, ctypes.byref(need))
    if rc:
        raise _err(rc, "admission conversion failed")
    return json.loads(buf.value.decode("utf-8"))


def _fast_or_noopinion(sar: dict) -> Tuple[int, str]:
    """Stores not loaded: fast paths still answer first (authorizer.go:38-57), else NoOpinion."""
    spec = sar.get("spec", {})
    name = spec.get("user", "")
    ra = spec.get("resourceAttributes") or {}
    ro = ra.get("verb", (spec.get("nonResourceAttributes") or {}).get("verb", "")) in ("get", "list", "watch")
    if name == "system:authorizer:cedar-authorizer" and ro and ra.get("group") == "cedar.k8s.aws" and ra.get("resource") == "policies":
        return 1, "cedar authorizer is always allowed to access policies"
    if name == "system:authorizer:cedar-authorizer" and ro and ra.get("group") == "rbac.authorization.k8s.io":
        return 1, "cedar authorizer is always allowed to read RBAC policies"
    return 2, ""
