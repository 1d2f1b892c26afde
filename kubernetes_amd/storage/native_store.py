"""ctypes binding of the native MVCC engine (native/store/mvcc_store.cc, libkamd_store.so).

Same interface as the pure-Python `MVCCStore` (so the API server can embed either), plus
`txn()` — etcd's multi-key Txn(If compares Then ops) under one revision. The engine is also
served by the `kamd-etcd` binary for multi-process API servers (`storage/remote.py`).
"""
from __future__ import annotations

import ctypes
import os
import struct
import threading

from ..native import LIB_DIR
from . import wire
from .mvcc import DELETE, PUT, CompactedError, Event, KV, TxnResult

_LIB = None


def _lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(LIB_DIR, "libkamd_store.so")
        if not os.path.exists(path):
            raise ImportError(f"{path} not built (python -m kubernetes_amd.native.build)")
        L = ctypes.CDLL(path)
        vp, cp, u32, i64 = ctypes.c_void_p, ctypes.c_char_p, ctypes.c_uint32, ctypes.c_int64
        outp, outl = ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(u32)
        L.kamd_store_open.restype = vp
        L.kamd_store_open.argtypes = [cp, ctypes.c_uint64]
        L.kamd_store_close.argtypes = [vp]
        L.kamd_store_rev.restype = i64
        L.kamd_store_rev.argtypes = [vp]
        L.kamd_store_compacted.restype = i64
        L.kamd_store_compacted.argtypes = [vp]
        L.kamd_store_size.restype = ctypes.c_uint64
        L.kamd_store_size.argtypes = [vp]
        L.kamd_store_txn.restype = ctypes.c_int
        L.kamd_store_txn.argtypes = [vp, cp, u32, ctypes.POINTER(i64)]
        L.kamd_store_get.restype = ctypes.c_int
        L.kamd_store_get.argtypes = [vp, cp, u32, outp, outl]
        L.kamd_store_range.restype = ctypes.c_int
        L.kamd_store_range.argtypes = [vp, cp, u32, u32, cp, u32, outp, outl]
        L.kamd_store_since.restype = ctypes.c_int
        L.kamd_store_since.argtypes = [vp, i64, cp, u32, outp, outl]
        L.kamd_store_compact.argtypes = [vp, i64]
        _LIB = L
    return _LIB


class NativeMVCCStore:
    def __init__(self, history: int = 200_000, wal_path: str | None = None):
        self._L = _lib()
        self._h = self._L.kamd_store_open(wal_path.encode() if wal_path else None, history)
        if not self._h:
            raise OSError(f"cannot open native store (wal={wal_path})")
        self._lock = threading.Lock()
        self._out = ctypes.c_void_p()
        self._outl = ctypes.c_uint32()

    # -- helpers ----------------------------------------------------------
    def _buf(self):
        return ctypes.string_at(self._out.value, self._outl.value) if self._outl.value else b""

    def _get(self, key):
        kb = key.encode()
        if not self._L.kamd_store_get(self._h, kb, len(kb), ctypes.byref(self._out), ctypes.byref(self._outl)):
            return None
        return wire.decode_kv(self._buf())[0]

    # -- public API (MVCCStore compatible) --------------------------------
    @property
    def revision(self) -> int:
        return self._L.kamd_store_rev(self._h)

    @property
    def compacted_revision(self) -> int:
        return self._L.kamd_store_compacted(self._h)

    def __len__(self):
        return self._L.kamd_store_size(self._h)

    def get(self, key):
        with self._lock:
            return self._get(key)

    def txn(self, cmps, ops) -> TxnResult:
        req = wire.encode_txn(cmps, ops)
        rev = ctypes.c_int64()
        with self._lock:
            r = self._L.kamd_store_txn(self._h, req, len(req), ctypes.byref(rev))
            if r == -2:
                raise ValueError("malformed txn")
            if r >= 0:
                return TxnResult(False, self._L.kamd_store_rev(self._h), r, self._get(cmps[r][1]))
            return TxnResult(True, rev.value)

    def create(self, key, value):
        with self._lock:
            res = self._txn_locked([(wire.CMP_ABSENT, key, 0, None)], [(wire.OP_PUT, key, value)])
            if res < 0:
                return None
            return Event(PUT, KV(key, value, res, res, 1), None)

    def update(self, key, value, expected_mod_rev):
        with self._lock:
            cur = self._get(key)
            if cur is None:
                return False, None
            if expected_mod_rev is not None and cur.mod_rev != expected_mod_rev:
                return False, cur
            res = self._txn_locked([(wire.CMP_MOD_REV, key, cur.mod_rev, None)], [(wire.OP_PUT, key, value)])
            return True, Event(PUT, KV(key, value, cur.create_rev, res, cur.version + 1), cur)

    def put(self, key, value):
        with self._lock:
            cur = self._get(key)
            res = self._txn_locked([], [(wire.OP_PUT, key, value)])
            if cur is None:
                return Event(PUT, KV(key, value, res, res, 1), None)
            return Event(PUT, KV(key, value, cur.create_rev, res, cur.version + 1), cur)

    def delete(self, key, expected_mod_rev=None):
        with self._lock:
            cur = self._get(key)
            if cur is None:
                return False, None
            if expected_mod_rev is not None and cur.mod_rev != expected_mod_rev:
                return False, cur
            res = self._txn_locked([(wire.CMP_MOD_REV, key, cur.mod_rev, None)], [(wire.OP_DELETE, key, None)])
            return True, Event(DELETE, KV(key, None, cur.create_rev, res, 0), cur)

    def _txn_locked(self, cmps, ops):
        req = wire.encode_txn(cmps, ops)
        rev = ctypes.c_int64()
        r = self._L.kamd_store_txn(self._h, req, len(req), ctypes.byref(rev))
        return rev.value if r == -1 else -1

    def range(self, prefix, limit=0, start_after=None):
        pb = prefix.encode()
        sb = (start_after or "").encode()
        with self._lock:
            self._L.kamd_store_range(self._h, pb, len(pb), limit, sb, len(sb), ctypes.byref(self._out),
                                     ctypes.byref(self._outl))
            return wire.decode_range(self._buf())

    def count(self, prefix):
        return len(self.range(prefix)[0])

    def events_since(self, rev, prefix=""):
        pb = prefix.encode()
        with self._lock:
            n = self._L.kamd_store_since(self._h, rev, pb, len(pb), ctypes.byref(self._out), ctypes.byref(self._outl))
            if n < 0:
                raise CompactedError(rev)
            buf = self._buf()
        (cnt,) = struct.unpack_from("<I", buf, 0)
        off = 4
        out = []
        for _ in range(cnt):
            t = buf[off]
            kv, off = wire.decode_kv(buf, off + 1)
            if t == 1:
                kv.value = None
            out.append(Event(DELETE if t == 1 else PUT, kv, None))
        return out

    def compact(self, rev):
        with self._lock:
            self._L.kamd_store_compact(self._h, rev)

    def close(self):
        if self._h:
            self._L.kamd_store_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
