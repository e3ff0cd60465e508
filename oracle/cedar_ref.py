"""ctypes binding of the C++ oracle (oracle/cedar_ref.cpp) — TEST INFRASTRUCTURE ONLY.

Used by tests/ (fast parity at sizes the Python oracle cannot reach), __graft_entry__.smoke() and
bench.py's `cpu_baseline` leg. The product never imports it. Build: `make -C oracle`.
"""
import ctypes
import json
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "_build", "libcedar_ref.so")

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"C++ oracle not built ({LIB_PATH}); run `make -C oracle`")
        L = ctypes.CDLL(LIB_PATH)
        P, sz = ctypes.c_void_p, ctypes.c_size_t
        L.cref_create.restype = P
        L.cref_destroy.argtypes = [P]
        L.cref_last_error.restype = ctypes.c_char_p
        L.cref_last_error.argtypes = [P]
        L.cref_add_tier.argtypes = [P]
        L.cref_add_document.argtypes = [P, ctypes.c_char_p, ctypes.c_char_p, sz, ctypes.c_char_p, ctypes.c_char_p]
        L.cref_add_policy.argtypes = [P, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, sz, ctypes.c_int]
        L.cref_set_entities.argtypes = [P, ctypes.c_char_p, sz]
        L.cref_load_items.argtypes = [P, ctypes.c_char_p, sz, ctypes.POINTER(ctypes.c_uint32)]
        L.cref_eval.argtypes = [P, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(sz)]
        L.cref_bench.argtypes = [P, ctypes.c_int, ctypes.c_double, ctypes.POINTER(ctypes.c_uint64),
                                 ctypes.POINTER(ctypes.c_double)]
        L.cref_free.argtypes = [P]
        _lib = L
    return _lib


class RefError(RuntimeError):
    pass


class RefPolicySet:
    """Tiered policy set (TieredPolicyStores restatement) evaluated by the C++ oracle."""

    def __init__(self):
        self.h = lib().cref_create()
        self._tier_open = False

    def close(self):
        if self.h:
            lib().cref_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def _chk(self, rc):
        if rc != 0:
            raise RefError(lib().cref_last_error(self.h).decode(errors="replace"))

    def set_entities(self, entities_json: str):
        """Static entities merged into every item's EntityMap (cedar_oracle.merge_static_entities)."""
        b = entities_json.encode() if entities_json else b""
        self._chk(lib().cref_set_entities(self.h, b, len(b)))

    def add_tier(self):
        self._chk(lib().cref_add_tier(self.h))

    def add_document(self, filename, text, id_prefix="policy", id_suffix=""):
        b = text.encode()
        self._chk(lib().cref_add_document(self.h, filename.encode(), b, len(b), id_prefix.encode(), id_suffix.encode()))

    def add_policy(self, policy_id, filename, text, zero_position=False):
        b = text.encode()
        self._chk(lib().cref_add_policy(self.h, policy_id.encode(), filename.encode(), b, len(b), int(zero_position)))

    @classmethod
    def from_stores(cls, stores, entities=None):
        """From cedargpu store objects (their `documents()` lists), one tier per store; `entities`:
        static entities (Cedar JSON list) merged into every EntityMap."""
        s = cls()
        if entities:
            s.set_entities(json.dumps(entities))
        for st in stores:
            s.add_tier()
            for d in st.documents():
                if d[0] == "doc":
                    _, fname, text, pre, suf = d
                    try:
                        s.add_document(fname, text, pre, suf)
                    except RefError:
                        # directory / CRD / AVP stores log and skip such a document (directory.go:69-73,
                        # crd.go:51-55,91-95, verified_permissions.go:89-93)
                        if not getattr(st, "skip_invalid", False):
                            raise
                else:
                    _, pid, fname, text, zero = d
                    s.add_policy(pid, fname, text, zero)
        return s

    def load_items(self, items_json: str) -> int:
        b = items_json.encode()
        n = ctypes.c_uint32(0)
        self._chk(lib().cref_load_items(self.h, b, len(b), ctypes.byref(n)))
        return n.value

    def evaluate(self, threads=8):
        """[(allow: bool, tier: int, diagnostic_json: str, reasons_json: str)] for the loaded items."""
        out = ctypes.c_void_p()
        n = ctypes.c_size_t(0)
        self._chk(lib().cref_eval(self.h, threads, ctypes.byref(out), ctypes.byref(n)))
        try:
            text = ctypes.string_at(out, n.value).decode()
        finally:
            lib().cref_free(out)
        res = []
        for line in text.split("\n")[:-1]:
            a, t, d, r = line.split("\t")
            res.append((a == "1", int(t), d, r))
        return res

    def bench(self, threads, seconds):
        """(decisions, wall seconds) over the loaded items on `threads` host threads."""
        d = ctypes.c_uint64(0)
        w = ctypes.c_double(0)
        self._chk(lib().cref_bench(self.h, threads, seconds, ctypes.byref(d), ctypes.byref(w)))
        return d.value, w.value


def items_json(items):
    """[(entities_json, request_json)] -> the JSON array the oracle loads."""
    return json.dumps([{"entities": e, "request": r} for e, r in items], separators=(",", ":"))
