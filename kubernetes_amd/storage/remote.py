"""asyncio client for the native store server (`kamd-etcd`) + a helper that runs one.

Several API server worker processes share one `kamd-etcd` (the role etcd plays for a set of
kube-apiservers, reference `staging/src/k8s.io/apiserver/pkg/storage/etcd3/store.go`): every
worker commits with compare-and-swap transactions and feeds its own watch cache from a single
ordered watch stream, so all workers observe the same revision order.

Requests are pipelined on one connection (ids matched to futures); watch events arrive on the
same connection as frames tagged with the watch id and are delivered synchronously to the
callback, in store order.
"""
from __future__ import annotations

import asyncio
import os
import struct
import subprocess
import tempfile
import time

from ..native import BIN_DIR
from . import wire
from .mvcc import CompactedError, TxnResult

_hdr = struct.Struct("<IIB")


class StoreError(Exception):
    pass


class _Proto(asyncio.Protocol):
    def __init__(self, owner):
        self.owner = owner
        self.buf = bytearray()
        self.transport = None

    def connection_made(self, transport):
        self.transport = transport

    def data_received(self, data):
        buf = self.buf
        buf += data
        off = 0
        n = len(buf)
        owner = self.owner
        while n - off >= 9:
            ln, rid, st = _hdr.unpack_from(buf, off)
            if n - off - 4 < ln:
                break
            payload = bytes(buf[off + 9:off + 4 + ln])
            off += 4 + ln
            owner._frame(rid, st, payload)
        if off:
            del buf[:off]

    def connection_lost(self, exc):
        self.owner._lost(exc)


class RemoteStore:
    def __init__(self, address: str):
        self.address = address
        self._proto = None
        self._next = 1
        self._pending: dict[int, asyncio.Future] = {}
        self._watches: dict[int, callable] = {}
        self._on_ok: dict[int, callable] = {}
        self._outbuf = None
        self.closed = False

    async def connect(self):
        loop = asyncio.get_running_loop()
        if self.address.startswith("unix://"):
            _, self._proto = await loop.create_unix_connection(lambda: _Proto(self), self.address[len("unix://"):])
        else:
            hp = self.address.split("://", 1)[-1]
            host, port = hp.rsplit(":", 1)
            _, self._proto = await loop.create_connection(lambda: _Proto(self), host, int(port))
        return self

    # -- framing ------------------------------------------------------------
    def _send(self, op, payload=b""):
        if self._proto is None or self.closed:
            raise StoreError("store connection closed")
        rid = self._next
        self._next += 1
        loop = asyncio.get_running_loop()
        fut = loop.create_future()
        self._pending[rid] = fut
        # requests issued in one event-loop iteration leave in ONE send (fewer syscalls under load)
        if self._outbuf is None:
            self._outbuf = [_hdr.pack(len(payload) + 5, rid, op), payload]
            loop.call_soon(self._flush)
        else:
            self._outbuf += (_hdr.pack(len(payload) + 5, rid, op), payload)
        return rid, fut

    def _flush(self):
        buf, self._outbuf = self._outbuf, None
        if buf and not self.closed and self._proto is not None:
            self._proto.transport.write(b"".join(buf))

    def _frame(self, rid, st, payload):
        if st == wire.EVENT:
            cb = self._watches.get(rid)
            if cb is not None:
                t = payload[0]
                kv, _ = wire.decode_kv(payload, 1)
                cb(t, kv)
            return
        if st == wire.PROGRESS:
            # excluded keys changed up to this revision (watch(..., exclude=...))
            cb = self._watches.get(rid)
            if cb is not None:
                cb(wire.PROGRESS, struct.unpack_from("<q", payload)[0])
            return
        cb = self._on_ok.pop(rid, None) if self._on_ok else None
        if cb is not None and st == wire.OK:
            # synchronous commit hook: runs before any later frame (e.g. the watch event of this
            # very commit) is processed
            cb(struct.unpack_from("<q", payload)[0])
        fut = self._pending.pop(rid, None)
        if fut is not None and not fut.done():
            fut.set_result((st, payload))

    def _lost(self, exc):
        self.closed = True
        for fut in self._pending.values():
            if not fut.done():
                fut.set_exception(StoreError(f"store connection lost: {exc}"))
        self._pending.clear()
        for cb in list(self._watches.values()):
            try:
                cb(None, None)  # stream end
            except Exception:
                pass
        self._watches.clear()

    # -- API ----------------------------------------------------------------
    async def txn(self, cmps, ops, on_ok=None) -> TxnResult:
        """on_ok(rev) is called synchronously when the commit reply arrives."""
        rid, fut = self._send(wire.TXN, wire.encode_txn(cmps, ops))
        if on_ok is not None:
            self._on_ok[rid] = on_ok
        st, p = await fut
        if st == wire.OK:
            return TxnResult(True, struct.unpack_from("<q", p)[0])
        if st == wire.FAILED:
            idx, kv, rev = wire.decode_failed(p)
            return TxnResult(False, rev, idx, kv)
        raise StoreError(f"txn failed with status {st}")

    async def get(self, key):
        kb = key.encode()
        _, fut = self._send(wire.GET, struct.pack("<I", len(kb)) + kb)
        st, p = await fut
        if st == wire.NOT_FOUND:
            return None
        return wire.decode_kv(p)[0]

    async def range(self, prefix, limit=0, start_after=None, revision=0):
        """(kvs, more, revision). `revision` > 0 reads the keys as they were at that revision
        (CompactedError below the retained history, StoreError for a future revision)."""
        if revision:
            payload = wire.encode_range(prefix, limit, start_after) + struct.pack("<q", revision)
            _, fut = self._send(wire.RANGE_AT, payload)
            st, p = await fut
            if st == wire.COMPACTED:
                raise CompactedError(revision)
            if st != wire.OK:
                raise StoreError(f"revision {revision} is a future revision" if st == wire.BAD and p else
                                 f"range at {revision} failed with status {st}")
            return wire.decode_range(p)
        _, fut = self._send(wire.RANGE, wire.encode_range(prefix, limit, start_after))
        st, p = await fut
        return wire.decode_range(p)

    async def revision(self):
        _, fut = self._send(wire.REV)
        st, p = await fut
        return struct.unpack_from("<q", p)[0]

    async def compact(self, rev):
        _, fut = self._send(wire.COMPACT, struct.pack("<q", rev))
        await fut

    async def watch(self, prefix, from_rev, callback, exclude=()):
        """callback(type, kv) for each event with mod_rev > from_rev (0 = only new events);
        callback(None, None) when the stream ends. Returns the store revision at subscribe.
        Keys under an `exclude` prefix are not delivered; instead callback(wire.PROGRESS, rev)
        reports (coalesced) that the store moved on to `rev`."""
        pb = prefix.encode()
        payload = struct.pack("<q", from_rev) + struct.pack("<I", len(pb)) + pb
        if exclude:
            payload += struct.pack("<H", len(exclude)) + b"".join(wire._s(x.encode()) for x in exclude)
        rid, fut = self._send(wire.WATCH, payload)
        # register before the reply: replayed events directly follow the OK frame
        self._watches[rid] = callback
        st, p = await fut
        if st == wire.COMPACTED:
            self._watches.pop(rid, None)
            raise CompactedError(from_rev)
        return struct.unpack_from("<q", p)[0]

    async def close(self):
        self.closed = True
        if self._proto is not None and self._proto.transport is not None:
            self._proto.transport.close()


class FanoutClient:
    """Hands an accepted watch connection to `kamd-etcd`'s watch fan-out (SCM_RIGHTS over the
    `<store socket>.watch` unix socket) with its spec; the store then serves the HTTP chunked
    watch stream itself (see native/store/mvcc_store.cc "Watch fan-out")."""

    LABEL, FIELD = 0, 1
    # "shard": key = the offset label, values = [count, index] (api/sharding.py)
    OPS = {"=": 0, "==": 0, "!=": 1, "in": 2, "notin": 3, "exists": 4, "!": 5, "shard": 6}

    def __init__(self, path):
        self.path = path

    @classmethod
    def for_store(cls, address):
        if address and address.startswith("unix://"):
            p = address[len("unix://"):] + ".watch"
            if os.path.exists(p):
                return cls(p)
        return None

    @staticmethod
    def _s(b: bytes) -> bytes:
        return struct.pack("<I", len(b)) + b

    def encode(self, prefix, send_initial, from_rev, timeout, reqs, protobuf=False) -> bytes:
        """reqs: [(target, op, key, [values])] with op one of OPS. Version 2 adds a trailing
        format byte: 1 = protobuf watch frames (`...protobuf;stream=watch`), 0 = JSON lines."""
        out = struct.pack("<BBqd", 2 if protobuf else 1, 1 if send_initial else 0, int(from_rev or 0),
                          float(timeout or 0))
        out += self._s(prefix.encode())
        out += struct.pack("<H", len(reqs))
        for target, op, key, vals in reqs:
            out += struct.pack("<BB", target, self.OPS[op]) + self._s(key.encode()) + struct.pack("<H", len(vals))
            for v in vals:
                out += self._s(str(v).encode())
        if protobuf:
            out += b"\x01"
        return struct.pack("<I", len(out)) + out

    def handoff(self, fd, msg: bytes):
        import socket
        s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        try:
            s.settimeout(5.0)
            s.connect(self.path)
            socket.send_fds(s, [msg], [fd])
        finally:
            s.close()


class StoreServer:
    """Runs `kamd-etcd` as a child process on a unix socket (or TCP port)."""

    def __init__(self, socket_path=None, wal=None, history=500_000, tcp=False, fan_threads=None):
        self.dir = None
        # watch fan-out threads in kamd-etcd (1..4); KAMD_ETCD_FAN_THREADS overrides the default 1
        self.fan_threads = int(fan_threads or os.environ.get("KAMD_ETCD_FAN_THREADS") or 1)
        if socket_path is None and not tcp:
            self.dir = tempfile.mkdtemp(prefix="kamd-etcd-")
            socket_path = os.path.join(self.dir, "store.sock")
        self.socket_path = socket_path
        self.tcp = tcp
        self.wal = wal
        self.history = history
        self.proc = None
        self.address = None

    def start(self, timeout=10.0):
        # KAMD_ETCD_BIN: run another build of the server (the ASan/UBSan one in
        # native/san/asan/ for the sanitizer tier); KAMD_ETCD_LOG_DIR: keep its stderr there
        exe = os.environ.get("KAMD_ETCD_BIN") or os.path.join(BIN_DIR, "kamd-etcd")
        if not os.path.exists(exe):
            raise StoreError(f"{exe} not built (python -m kubernetes_amd.native.build)")
        from ..api.protobuf import SCHEMA_PATH
        cmd = [exe, "--history", str(self.history), "--fan-threads", str(self.fan_threads)]
        if os.path.exists(SCHEMA_PATH):
            cmd += ["--pb-schema", SCHEMA_PATH]     # the fan-out transcodes protobuf values for JSON watchers
        port_file = None
        if self.tcp:
            port_file = tempfile.mktemp(prefix="kamd-etcd-port-")
            cmd += ["--listen-tcp", "0", "--port-file", port_file]
        else:
            # watch fan-out handoffs next to the store socket (FanoutClient.for_store)
            cmd += ["--listen-unix", self.socket_path, "--listen-handoff", self.socket_path + ".watch"]
        if self.wal:
            cmd += ["--wal", self.wal]
        log_dir = os.environ.get("KAMD_ETCD_LOG_DIR")
        err = subprocess.DEVNULL
        if log_dir:
            os.makedirs(log_dir, exist_ok=True)
            err = open(os.path.join(log_dir, f"kamd-etcd.{os.getpid()}.{id(self)}.log"), "ab")
        self.proc = subprocess.Popen(cmd, stdout=subprocess.DEVNULL, stderr=err, start_new_session=True)
        if err is not subprocess.DEVNULL:
            err.close()
        deadline = time.time() + timeout
        while time.time() < deadline:
            if self.proc.poll() is not None:
                raise StoreError(f"kamd-etcd exited with {self.proc.returncode}")
            if self.tcp and os.path.exists(port_file) and os.path.getsize(port_file):
                with open(port_file) as f:
                    self.address = f"tcp://127.0.0.1:{int(f.read())}"
                os.unlink(port_file)
                return self.address
            # both sockets: an API server probing the fan-out socket right after start() must find
            # it (a slow start, e.g. the TSan build, used to leave it missing)
            if not self.tcp and os.path.exists(self.socket_path) and os.path.exists(self.socket_path + ".watch"):
                self.address = f"unix://{self.socket_path}"
                return self.address
            time.sleep(0.01)
        raise StoreError("kamd-etcd did not start")

    def stop(self):
        if self.proc and self.proc.poll() is None:
            self.proc.terminate()
            try:
                self.proc.wait(5)
            except subprocess.TimeoutExpired:
                self.proc.kill()
                self.proc.wait()
        if self.dir:
            try:
                for p in (self.socket_path, self.socket_path + ".watch"):
                    if os.path.exists(p):
                        os.unlink(p)
                os.rmdir(self.dir)
            except OSError:
                pass
