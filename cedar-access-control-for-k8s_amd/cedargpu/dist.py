"""Multi-GPU serving: request sharding and RCCL hot-reload of the compiled image.

One process per GPU (torchrun). Decisions are independent, so requests shard across GPUs with no
collective on the decision path; every GPU holds a replica of the immutable policy image. On a
policy reload, the moment where the reference swaps its `*cedar.PolicySet`
(internal/server/store/directory.go:81, verified_permissions.go:99; in-place mutation at
crd.go:62,85,102,114), one rank compiles the new tiers and `broadcast_image` ships the blob to every
GPU with one RCCL broadcast (`cg_broadcast_image`), after which each rank activates the new epoch.

torch.distributed is plumbing here: it exchanges the 128-byte RCCL id over whatever process group
the caller runs (gloo on CPU tensors is enough).
"""
from __future__ import annotations

import ctypes
from typing import Optional, Tuple

from ._lib import DeviceError, _err, lib

_P = ctypes.c_void_p
UNIQUE_ID_BYTES = 128


def shard(n: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous request range [start, stop) of `rank` among `world` (sizes differ by at most 1)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank / world")
    q, r = divmod(n, world)
    start = rank * q + min(rank, r)
    return start, start + q + (1 if rank < r else 0)


def unique_id() -> bytes:
    buf = ctypes.create_string_buffer(UNIQUE_ID_BYTES)
    rc = lib.cg_comm_unique_id(buf, UNIQUE_ID_BYTES)
    if rc:
        raise DeviceError(rc, "ncclGetUniqueId failed: " + lib.cg_comm_last_error(None).decode())
    return buf.raw


def exchange_unique_id(rank: int, make=unique_id, group=None) -> bytes:
    """Rank 0 makes the RCCL id; torch.distributed broadcasts it to every rank."""
    import torch.distributed as dist
    obj = [make() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0, group=group)
    return obj[0]


class Comm:
    """An RCCL communicator over the GPUs of one node (one rank per GPU)."""

    def __init__(self, device: int, world: int, rank: int, uid: bytes):
        self.rank, self.world = rank, world
        self._h = _P()
        rc = lib.cg_comm_create(device, world, rank, uid, len(uid), ctypes.byref(self._h))
        if rc:
            raise DeviceError(rc, "RCCL communicator: " + lib.cg_comm_last_error(None).decode())

    def close(self):
        if self._h:
            lib.cg_comm_destroy(self._h)
            self._h = _P()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def broadcast_image(self, ctx, image: Optional[bytes], epoch: int, root: int = 0, activate: bool = True) -> int:
        """Collective: root's compiled image reaches every rank's ctx as `epoch`. Returns its size."""
        n = ctypes.c_size_t(0)
        # the bytes object's own buffer (no copy of a 100 MB image; the library only reads it)
        buf = ctypes.cast(ctypes.c_char_p(image), ctypes.c_void_p) if image is not None else None
        rc = lib.cg_broadcast_image(ctx._h, self._h, root, buf, len(image) if image is not None else 0, epoch,
                                    1 if activate else 0, ctypes.byref(n))
        if rc:
            raise _err(rc, "image broadcast: " + lib.cg_comm_last_error(self._h).decode())
        return n.value

    def broadcast_delta(self, ctx, base_epoch: int, delta: Optional[bytes], epoch: int, root: int = 0,
                        activate: bool = True) -> int:
        """Collective: root's delta image against `base_epoch` is applied on every rank's GPU as
        `epoch` (activated only when every rank applied it). Returns the delta's size."""
        n = ctypes.c_size_t(0)
        buf = ctypes.cast(ctypes.c_char_p(delta), ctypes.c_void_p) if delta is not None else None
        rc = lib.cg_broadcast_delta(ctx._h, self._h, root, base_epoch, buf, len(delta) if delta is not None else 0,
                                    epoch, 1 if activate else 0, ctypes.byref(n))
        if rc:
            raise _err(rc, "delta broadcast: " + lib.cg_comm_last_error(self._h).decode())
        return n.value
