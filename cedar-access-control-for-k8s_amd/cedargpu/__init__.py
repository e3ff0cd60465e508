"""cedargpu — Python binding of the MI355X Cedar evaluator C-ABI (include/cedargpu.h).

Mirrors the reference's store interface for the hot path:
  * `MemoryStore` / `DirectoryStore` / `CRDStore` / `AVPStore` / `StaticStore` — policy sources
    with the reference's policy-ID conventions (internal/server/store/*.go);
  * `TieredPolicyStores.is_authorized(entities, request)` — internal/server/store/store.go:25-42,
    evaluated on the GPU; `is_authorized_batch` evaluates many requests in one launch.
The product path has no CPU fallback: importing this package fails loudly when libcedargpu.so
is missing, and evaluation raises `DeviceError` when no GPU is present.
"""
from ._lib import CedarGPUError, CompileError, DeadlineError, DeviceError, lib, lib_path  # noqa: F401
from .store import (ALLOW_ALL_ADMISSION, FAULT_BAD_KIDX, FAULT_DEVICE_ERROR, FAULT_NONE, FAULT_STALL, AdmissionHandler,  # noqa: F401
                    Authorizer, AVPStore, Batch, Compiler, Context, CRDStore, DirectoryStore, MemoryStore, PolicyStore,
                    Queue, StaticStore, TieredPolicyStores, admission_to_cedar_json, atomic_policies, build_image,
                    delta_info, device_count, image_delta, image_patch, image_stats, index_stats, pinned_stats)
from .store import (ROUTE_CLASS, ROUTE_FIRST_SLOT, ROUTE_FU_BIG, ROUTE_FU_GEN, ROUTE_FU_OVF, ROUTE_RERUN)  # noqa: F401
