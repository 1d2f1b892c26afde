"""Embedded MVCC key-value store with etcd-v3 semantics (pure-Python engine).

What the API server needs from etcd (reference `staging/src/k8s.io/apiserver/pkg/storage/etcd3/store.go:128-666`):
  * a single monotonically increasing cluster revision,
  * per-key create/mod revision and version,
  * compare-and-swap on mod revision (GuaranteedUpdate / conditional delete),
  * ordered range reads with limit + continue key (list chunking),
  * a history of events since a revision (watch), with compaction.

The same interface is implemented natively in C++ (`native/store/mvcc_store.cc`, loaded by
`kubernetes_amd.storage.native_store`); `open_store()` picks the native engine when built.
"""
from __future__ import annotations

import bisect
import os
import struct
import threading
from collections import deque

PUT, DELETE = 0, 1


class CompactedError(Exception):
    """Requested revision is older than the compacted history (HTTP 410 Gone)."""


class KV:
    __slots__ = ("key", "value", "create_rev", "mod_rev", "version")

    def __init__(self, key, value, create_rev, mod_rev, version):
        self.key, self.value, self.create_rev, self.mod_rev, self.version = key, value, create_rev, mod_rev, version


class Event:
    __slots__ = ("type", "kv", "prev")

    def __init__(self, type_, kv, prev):
        self.type, self.kv, self.prev = type_, kv, prev


class TxnResult:
    __slots__ = ("ok", "rev", "failed", "current")

    def __init__(self, ok, rev, failed=-1, current=None):
        self.ok, self.rev, self.failed, self.current = ok, rev, failed, current


class MVCCStore:
    """Thread-safe; all mutations are serialized under one lock like etcd's apply loop."""

    def __init__(self, history: int = 200_000, wal_path: str | None = None):
        self._lock = threading.Lock()
        self._data: dict[str, KV] = {}
        self._keys: list[str] = []          # sorted key index for range scans
        self._rev = 1                       # etcd starts at revision 1
        self._compact_rev = 0
        self._history: deque[Event] = deque()
        self._history_cap = history
        self._wal = None
        if wal_path:
            self._replay(wal_path)
            self._wal = open(wal_path, "ab", buffering=0)

    # -- durability: simple append-only WAL (length-prefixed records) ----
    def _log(self, op, key, value):
        if self._wal is None:
            return
        kb = key.encode()
        rec = struct.pack("<BII", op, len(kb), len(value or b"")) + kb + (value or b"")
        self._wal.write(rec)

    def _replay(self, path):
        if not os.path.exists(path):
            return
        with open(path, "rb") as f:
            buf = f.read()
        off = 0
        while off + 9 <= len(buf):
            op, kl, vl = struct.unpack_from("<BII", buf, off)
            off += 9
            if off + kl + vl > len(buf):
                break  # torn tail write
            key = buf[off:off + kl].decode()
            val = buf[off + kl:off + kl + vl]
            off += kl + vl
            if op == PUT:
                self._apply_put(key, val)
            else:
                self._apply_delete(key)

    # -- internals --------------------------------------------------------
    def _record(self, ev):
        self._history.append(ev)
        if len(self._history) > self._history_cap:
            old = self._history.popleft()
            self._compact_rev = old.kv.mod_rev

    def _apply_put(self, key, value, rev=None):
        if rev is None:
            self._rev += 1
            rev = self._rev
        prev = self._data.get(key)
        if prev is None:
            kv = KV(key, value, rev, rev, 1)
            bisect.insort(self._keys, key)
        else:
            kv = KV(key, value, prev.create_rev, rev, prev.version + 1)
        self._data[key] = kv
        ev = Event(PUT, kv, prev)
        self._record(ev)
        return ev

    def _apply_delete(self, key, rev=None, tombstone=None):
        prev = self._data.pop(key, None)
        if prev is None:
            return None
        if rev is None:
            self._rev += 1
            rev = self._rev
        i = bisect.bisect_left(self._keys, key)
        del self._keys[i]
        ev = Event(DELETE, KV(key, tombstone, prev.create_rev, rev, 0), prev)
        self._record(ev)
        return ev

    # -- public API -------------------------------------------------------
    @property
    def revision(self) -> int:
        return self._rev

    @property
    def compacted_revision(self) -> int:
        return self._compact_rev

    def get(self, key: str) -> KV | None:
        return self._data.get(key)

    def create(self, key: str, value: bytes):
        """Txn(If(mod_revision(key)==0) Then(Put)). Returns Event or None if exists."""
        with self._lock:
            if key in self._data:
                return None
            self._log(PUT, key, value)
            return self._apply_put(key, value)

    def update(self, key: str, value: bytes, expected_mod_rev: int | None):
        """CAS put. Returns (ok, Event|current KV)."""
        with self._lock:
            cur = self._data.get(key)
            if cur is None:
                return False, None
            if expected_mod_rev is not None and cur.mod_rev != expected_mod_rev:
                return False, cur
            self._log(PUT, key, value)
            return True, self._apply_put(key, value)

    def put(self, key: str, value: bytes):
        with self._lock:
            self._log(PUT, key, value)
            return self._apply_put(key, value)

    def delete(self, key: str, expected_mod_rev: int | None = None):
        with self._lock:
            cur = self._data.get(key)
            if cur is None:
                return False, None
            if expected_mod_rev is not None and cur.mod_rev != expected_mod_rev:
                return False, cur
            self._log(DELETE, key, None)
            return True, self._apply_delete(key)

    def txn(self, cmps, ops):
        """etcd Txn(If cmps Then ops) under ONE revision; same encoding as `storage.wire`
        (cmps: (kind, key, arg, value); ops: (kind, key, value[, rv_token])). Returns a
        `TxnResult`-like object: ok, rev, failed (index of the first false compare), current."""
        with self._lock:
            for i, (kind, key, arg, val) in enumerate(cmps):
                cur = self._data.get(key)
                ok = ((cur.mod_rev == arg if cur else arg == 0) if kind == 0 else
                      cur is not None if kind == 1 else cur is None if kind == 2 else
                      cur is not None and cur.value == val)
                if not ok:
                    return TxnResult(False, self._rev, i, cur)
            rev = self._rev + 1
            rs = str(rev).encode()
            changed = False
            for op in ops:
                kind, key, val = op[0], op[1], op[2]
                if kind >= 2 and val is not None:
                    val = val.replace(op[3], rs)
                if kind in (0, 2):
                    self._log(PUT, key, val)
                    self._apply_put(key, val, rev)
                    changed = True
                elif key in self._data:
                    self._log(DELETE, key, None)
                    self._apply_delete(key, rev, val if kind == 3 else None)
                    changed = True
            if changed:
                self._rev = rev
            return TxnResult(True, self._rev)

    def range(self, prefix: str, limit: int = 0, start_after: str | None = None):
        """Returns (list[KV], more: bool, revision)."""
        with self._lock:
            lo = bisect.bisect_right(self._keys, start_after) if start_after else bisect.bisect_left(self._keys, prefix)
            out = []
            keys = self._keys
            n = len(keys)
            i = lo
            while i < n:
                k = keys[i]
                if not k.startswith(prefix):
                    break
                if limit and len(out) >= limit:
                    return out, True, self._rev
                out.append(self._data[k])
                i += 1
            return out, False, self._rev

    def count(self, prefix: str) -> int:
        with self._lock:
            lo = bisect.bisect_left(self._keys, prefix)
            hi = bisect.bisect_left(self._keys, prefix + "\xff")
            return hi - lo

    def events_since(self, rev: int, prefix: str = ""):
        """Events with mod_rev > rev (watch replay). Raises CompactedError."""
        with self._lock:
            if rev < self._compact_rev:
                raise CompactedError(rev)
            # history is revision ordered; binary search on mod_rev
            h = self._history
            lo, hi = 0, len(h)
            while lo < hi:
                mid = (lo + hi) // 2
                if h[mid].kv.mod_rev <= rev:
                    lo = mid + 1
                else:
                    hi = mid
            return [e for e in list(h)[lo:] if e.kv.key.startswith(prefix)]

    def compact(self, rev: int):
        with self._lock:
            while self._history and self._history[0].kv.mod_rev <= rev:
                self._history.popleft()
            self._compact_rev = max(self._compact_rev, rev)

    def close(self):
        if self._wal:
            self._wal.close()
            self._wal = None
