"""ctypes loader for libcedargpu.so (built in-tree by csrc/Makefile). Fails loudly if missing."""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
lib_path = os.path.join(_HERE, "libcedargpu.so")
# Host sanitizer runs only (tools/sanitize.sh): the ASan build of the host engine over the
# host-memory device stand-in (csrc/device_stub.cpp), for the CPU tests. It has no GPU path.
SANITIZER_BUILD = bool(os.environ.get("CEDARGPU_SANITIZER_LIB"))
if SANITIZER_BUILD:
    lib_path = os.environ["CEDARGPU_SANITIZER_LIB"]
# A/B studies only (tools/ab_lib.sh): another build of this library, e.g. an earlier commit's, run
# by the same bench in the same GPU session; symbols it predates are left unbound.
AB_BUILD = bool(os.environ.get("CEDARGPU_AB_LIB"))
if AB_BUILD:
    lib_path = os.environ["CEDARGPU_AB_LIB"]

if not os.path.exists(lib_path):
    raise ImportError(f"cedargpu: native library not built ({lib_path}); run `make -C cedar-access-control-for-k8s_amd/csrc`"
                      " or __graft_entry__.build()")

lib = ctypes.CDLL(lib_path)

CG_OK = 0
CG_E_ARG, CG_E_PARSE, CG_E_COMPILE, CG_E_STATE, CG_E_DEVICE, CG_E_TIMEOUT, CG_E_RANGE = -1, -2, -3, -4, -5, -6, -7


class CedarGPUError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"cedargpu error {code}: {msg}")
        self.code = code
        self.msg = msg


class CompileError(CedarGPUError):
    pass


class DeviceError(CedarGPUError):
    pass


class DeadlineError(CedarGPUError):
    """CG_E_TIMEOUT: the call's deadline passed (callers fail safe as on a webhook timeout)."""


def _err(code, msg):
    if code in (CG_E_PARSE, CG_E_COMPILE):
        return CompileError(code, msg)
    if code == CG_E_DEVICE:
        return DeviceError(code, msg)
    if code == CG_E_TIMEOUT:
        return DeadlineError(code, msg)
    return CedarGPUError(code, msg)


P = ctypes.c_void_p
u32, u64, i64, sz = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int64, ctypes.c_size_t
cstr = ctypes.c_char_p

_SIGS = {
    "cg_version": (cstr, []),
    "cg_free": (None, [P]),
    "cg_compiler_create": (ctypes.c_int, [ctypes.POINTER(P)]),
    "cg_compiler_destroy": (None, [P]),
    "cg_compiler_last_error": (cstr, [P]),
    "cg_compiler_add_tier": (ctypes.c_int, [P]),
    "cg_compiler_clear": (ctypes.c_int, [P]),
    "cg_compiler_cache_stats": (ctypes.c_int, [P, ctypes.POINTER(u64), ctypes.POINTER(u64), ctypes.POINTER(u64)]),
    "cg_compiler_add_document": (ctypes.c_int, [P, cstr, cstr, sz, cstr, cstr]),
    "cg_compiler_add_policy": (ctypes.c_int, [P, cstr, cstr, cstr, sz, ctypes.c_int]),
    "cg_compiler_set_entities": (ctypes.c_int, [P, cstr, sz]),
    "cg_compiler_set_incremental": (ctypes.c_int, [P, ctypes.c_int]),
    "cg_compiler_last_build": (ctypes.c_int, [P, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(u64), ctypes.POINTER(u64),
                                              ctypes.POINTER(ctypes.c_char_p)]),
    "cg_compiler_add_document_ex": (ctypes.c_int, [P, cstr, cstr, sz, cstr, cstr, ctypes.c_int]),
    "cg_compiler_doc_errors": (ctypes.c_int, [P, P, sz, ctypes.POINTER(sz)]),
    "cg_compiler_build": (ctypes.c_int, [P, u64, ctypes.POINTER(P), ctypes.POINTER(sz)]),
    "cg_compiler_build_sized": (ctypes.c_int, [P, u64, ctypes.POINTER(sz)]),
    "cg_compiler_write_image": (ctypes.c_int, [P, P, sz]),
    "cg_image_info": (ctypes.c_int, [P, sz, ctypes.POINTER(u32), ctypes.POINTER(u32), ctypes.POINTER(u64)]),
    "cg_image_stats": (ctypes.c_int, [P, sz] + [ctypes.POINTER(u32)] * 4),
    "cg_image_policy_atomic": (ctypes.c_int, [P, sz, u32, ctypes.POINTER(ctypes.c_int)]),
    "cg_image_indexed": (ctypes.c_int, [P, sz, ctypes.POINTER(ctypes.c_int)]),
    "cg_image_index_stats": (ctypes.c_int, [P, sz] + [ctypes.POINTER(u32)] * 6),
    "cg_image_like_slots": (ctypes.c_int, [P, sz] + [ctypes.POINTER(u32)] * 2),
    "cg_device_count": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
    "cg_device_synchronize": (ctypes.c_int, [ctypes.c_int]),
    "cg_ctx_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(P)]),
    "cg_ctx_destroy": (None, [P]),
    "cg_last_error": (cstr, [P]),
    "cg_ctx_inject_fault": (ctypes.c_int, [P, ctypes.c_int, u64]),
    "cg_pinned_stats": (ctypes.c_int, [ctypes.POINTER(u64), ctypes.POINTER(u64), ctypes.POINTER(u64)]),
    "cg_image_load": (ctypes.c_int, [P, P, sz, u64]),
    "cg_image_load_device": (ctypes.c_int, [P, P, sz, u64, P]),
    "cg_image_load_peer": (ctypes.c_int, [P, P, u64]),
    "cg_image_delta": (ctypes.c_int, [P, sz, P, sz, ctypes.POINTER(P), ctypes.POINTER(sz)]),
    "cg_image_patch": (ctypes.c_int, [P, sz, P, sz, ctypes.POINTER(P), ctypes.POINTER(sz)]),
    "cg_delta_info": (ctypes.c_int, [P, sz] + [ctypes.POINTER(u64)] * 4),
    "cg_image_load_delta": (ctypes.c_int, [P, u64, P, sz, u64]),
    "cg_image_activate": (ctypes.c_int, [P, u64]),
    "cg_image_active": (ctypes.c_int, [P, ctypes.POINTER(u64)]),
    "cg_image_unload": (ctypes.c_int, [P, u64]),
    "cg_comm_unique_id": (ctypes.c_int, [P, sz]),
    "cg_comm_create": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, P, sz, ctypes.POINTER(P)]),
    "cg_comm_destroy": (None, [P]),
    "cg_comm_last_error": (cstr, [P]),
    "cg_broadcast_image": (ctypes.c_int, [P, P, ctypes.c_int, P, sz, u64, ctypes.c_int, ctypes.POINTER(sz)]),
    "cg_broadcast_delta": (ctypes.c_int, [P, P, ctypes.c_int, u64, P, sz, u64, ctypes.c_int, ctypes.POINTER(sz)]),
    "cg_batch_create": (ctypes.c_int, [P, ctypes.POINTER(P)]),
    "cg_batch_destroy": (None, [P]),
    "cg_batch_add_json": (ctypes.c_int, [P, cstr, sz]),
    "cg_batch_size": (u32, [P]),
    "cg_batch_submit": (ctypes.c_int, [P]),
    "cg_batch_wait": (ctypes.c_int, [P, i64]),
    "cg_batch_set_profile": (ctypes.c_int, [P, ctypes.c_int]),
    "cg_batch_profile": (ctypes.c_int, [P, ctypes.POINTER(ctypes.c_double), ctypes.c_size_t]),
    "cg_batch_decision": (ctypes.c_int, [P, u32, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(u32)]),
    "cg_batch_diagnostic": (ctypes.c_int, [P, u32, ctypes.c_int, P, sz, ctypes.POINTER(sz)]),
    "cg_batch_reasons": (ctypes.c_int, [P, u32, ctypes.POINTER(u32), u32, ctypes.POINTER(u32), ctypes.POINTER(u32)]),
    "cg_batch_time": (ctypes.c_int, [P, u32, ctypes.POINTER(ctypes.c_float)]),
    "cg_batch_time_split": (ctypes.c_int, [P, u32, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float)]),
    "cg_batch_reruns": (ctypes.c_int, [P, ctypes.POINTER(u32)]),
    "cg_batch_route": (ctypes.c_int, [P, u32, ctypes.POINTER(u32), ctypes.POINTER(u32)]),
    "cg_batch_followups": (ctypes.c_int, [P, ctypes.POINTER(u32)]),
    "cg_batch_bytes": (ctypes.c_int, [P, ctypes.POINTER(u64), ctypes.POINTER(u64), ctypes.POINTER(u64)]),
    "cg_batch_io": (ctypes.c_int, [P] + [ctypes.POINTER(ctypes.c_uint64)] * 4),
    "cg_batch_add_sar_json": (ctypes.c_int, [P, cstr, sz]),
    "cg_sar_to_cedar_json": (ctypes.c_int, [cstr, sz, P, sz, ctypes.POINTER(sz)]),
    "cg_batch_authz": (ctypes.c_int, [P, u32, ctypes.POINTER(ctypes.c_int), P, sz, ctypes.POINTER(sz)]),
    "cg_is_authorized_json": (ctypes.c_int, [P, cstr, sz, ctypes.POINTER(ctypes.c_int), P, sz, ctypes.POINTER(sz)]),
    "cg_encode_sar_check": (ctypes.c_int, [P, sz, cstr, sz, ctypes.POINTER(u32), ctypes.POINTER(u32),
                                           ctypes.POINTER(u32), ctypes.POINTER(i64)]),
    "cg_encode_items_check": (ctypes.c_int, [P, sz, cstr, sz, ctypes.POINTER(u32), ctypes.POINTER(u32),
                                             ctypes.POINTER(i64)]),
    "cg_json_split_check": (ctypes.c_int, [cstr, sz, u32, ctypes.POINTER(i64), ctypes.POINTER(ctypes.c_int)]),
    "cg_batch_add_admission_json": (ctypes.c_int, [P, cstr, sz]),
    "cg_batch_admit": (ctypes.c_int, [P, u32, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int), P, sz,
                                      ctypes.POINTER(sz)]),
    "cg_admission_to_cedar_json": (ctypes.c_int, [cstr, sz, P, sz, ctypes.POINTER(sz)]),
    "cg_queue_create_multi": (ctypes.c_int, [ctypes.POINTER(P), u32, u32, u32, ctypes.POINTER(P)]),
    "cg_queue_gpu_stats": (ctypes.c_int, [P, u32, ctypes.POINTER(u64), ctypes.POINTER(u64)]),
    "cg_queue_create": (ctypes.c_int, [P, u32, u32, ctypes.POINTER(P)]),
    "cg_queue_destroy": (None, [P]),
    "cg_queue_last_error": (cstr, []),
    "cg_queue_authorize_sar": (ctypes.c_int, [P, cstr, sz, i64, ctypes.POINTER(ctypes.c_int), P, sz, ctypes.POINTER(sz)]),
    "cg_queue_is_authorized_json": (ctypes.c_int, [P, cstr, sz, i64, ctypes.POINTER(ctypes.c_int), P, sz,
                                                   ctypes.POINTER(sz)]),
    "cg_queue_dropped": (ctypes.c_int, [P, ctypes.POINTER(ctypes.c_uint64)]),
    "cg_queue_stats": (ctypes.c_int, [P] + [ctypes.POINTER(u64)] * 5),
    "cg_queue_metrics_get": (ctypes.c_int, [P, P, sz]),
    "cg_metrics_latency_bounds": (ctypes.POINTER(u64), [ctypes.POINTER(u32)]),
    "cg_queue_loadgen": (ctypes.c_int, [P, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(sz), u32, u32, u64,
                                        ctypes.POINTER(ctypes.c_double), ctypes.POINTER(u64), ctypes.POINTER(u64),
                                        ctypes.POINTER(u64), ctypes.POINTER(u64)]),
    "cg_queue_loadgen_n": (ctypes.c_int, [P, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(sz), u32, u32, u32, u64,
                                          ctypes.POINTER(ctypes.c_double), ctypes.POINTER(u64), ctypes.POINTER(u64),
                                          ctypes.POINTER(u64), ctypes.POINTER(u64)]),
    "cg_queue_authorize_sar_n": (ctypes.c_int, [P, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(sz), u32, i64,
                                                ctypes.POINTER(ctypes.c_int), P, sz, ctypes.POINTER(sz), ctypes.POINTER(sz)]),
}

for _name, (_res, _args) in _SIGS.items():
    if AB_BUILD and not hasattr(lib, _name):
        continue
    _f = getattr(lib, _name)  # AttributeError here = the library does not export a declared symbol
    _f.restype = _res
    _f.argtypes = _args

EXPORTED = tuple(_SIGS)
