"""etcd v3 client storage backend: the API server's store interface over any etcd v3 endpoint.

Parity: `staging/src/k8s.io/apiserver/pkg/storage/etcd3/store.go:128-666` — the reference API
server is an etcd v3 client: Create / GuaranteedUpdate are `Txn(If ModRevision(key) == rev ...)`
(`:152,263`), List is a prefix Range (`:428`), Watch is a Watch stream from `rv + 1` with
`prev_kv` so that DELETE events carry the deleted object (`watcher.go`), the resourceVersion is
the key's ModRevision. `Etcd3Store` exposes exactly the interface of `storage.remote.RemoteStore`
(txn / get / range / revision / compact / watch / close), so an API server pointed at
`--etcd-servers=http://HOST:2379` (or https with `--etcd-cafile/--etcd-certfile/--etcd-keyfile`)
runs against a real etcd cluster — or against `kamd-etcd-gateway`, the etcd v3 front of the
native store — with no other change.

Mapping of the native store's transaction language onto etcd v3:
  * compares: MOD_REV(key, r) -> ModRevision(key) == r (r == 0: the key is absent);
    EXISTS -> Version(key) > 0; ABSENT -> Version(key) == 0; VALUE -> Value(key) == v;
  * ops: PUT / DELETE as such; PUT_INJECT (JSON storage: the value carries the API server's
    secret resourceVersion token) stores the value without the token, behind a header that
    records where it stood; every read splices the key's ModRevision back in at those offsets —
    the reference never stores the resourceVersion either. Only values that carry the header
    are rewritten: object content (an annotation, a protobuf string) is never touched, so no
    user-chosen text can change what another value decodes to; DELETE_TOMBSTONE
    deletes (the watch's prev_kv is the deleted object);
  * a failed Txn reports which compare failed and that key's current value: the failure branch
    reads every compared key and the compares are re-evaluated on what it returned;
  * the commit hook `on_ok(rev)` runs when the Txn response arrives (etcd orders nothing between
    a Txn response and a watch event; the API server tolerates either order);
  * `watch(..., exclude=...)`: events under excluded prefixes are reported as progress only.
Several endpoints (comma-separated) are tried in order until one answers (clientv3 balancer).
Keys may live under a namespace prefix (`--etcd-prefix`, the etcd `--namespace` idea).
"""
from __future__ import annotations

import asyncio
import logging
from urllib.parse import urlparse

import grpc

from . import wire
from .etcdv3 import M, PKG, SERVICES, prefix_end, T_VERSION, T_MOD, T_VALUE, EQUAL, GREATER
from .mvcc import KV, CompactedError, TxnResult

log = logging.getLogger("etcd3-client")

# PUT_INJECT values: INJECT_MAGIC | u16 n | n x u32 offset | value with the n tokens removed
INJECT_MAGIC = b"\x00KRV"
_PAGE = 10_000
_OPTS = [("grpc.max_receive_message_length", 1 << 30), ("grpc.max_send_message_length", 1 << 30)]


class Etcd3Error(Exception):
    pass


def is_etcd3_address(address: str) -> bool:
    return isinstance(address, str) and address.split("://", 1)[0] in ("http", "https", "etcd3")


def _creds(tls):
    cafile, certfile, keyfile = tls or (None, None, None)

    def rd(p):
        if not p:
            return None
        with open(p, "rb") as f:
            return f.read()
    return grpc.ssl_channel_credentials(root_certificates=rd(cafile), private_key=rd(keyfile),
                                        certificate_chain=rd(certfile))


class Etcd3Store:
    """`address`: `http(s)://host:port[,http(s)://host2:port2...][#/namespace]`."""

    def __init__(self, address: str, tls=None, namespace: str | None = None):
        spec, _, frag = address.partition("#")
        self.endpoints = [e.strip() for e in spec.split(",") if e.strip()]
        self.namespace = (namespace if namespace is not None else frag).rstrip("/")
        self.tls = tls
        self.channel = None
        self.target = None
        self.closed = False
        self._watch_tasks: set = set()

    # -- connection ---------------------------------------------------------------------------
    def _stubs(self, channel):
        for svc, methods in SERVICES.items():
            for name, (req, resp, kind) in methods.items():
                path = f"/{PKG}.{svc}/{name}"
                mk = channel.stream_stream if kind == "stream" else channel.unary_unary
                setattr(self, "_" + name, mk(path, request_serializer=M[req].SerializeToString,
                                              response_deserializer=M[resp].FromString))

    async def connect(self, timeout=10.0):
        errs = []
        for ep in self.endpoints:
            u = urlparse(ep if "://" in ep else "http://" + ep)
            target = u.netloc or u.path
            ch = (grpc.aio.secure_channel(target, _creds(self.tls), options=_OPTS) if u.scheme == "https"
                  else grpc.aio.insecure_channel(target, options=_OPTS))
            self._stubs(ch)
            try:
                await self._Status(M["StatusRequest"](), timeout=timeout)
            except grpc.aio.AioRpcError as e:
                errs.append(f"{ep}: {e.code().name} {e.details()}")
                await ch.close()
                continue
            self.channel, self.target = ch, ep
            return self
        raise Etcd3Error("no etcd endpoint answered: " + "; ".join(errs))

    async def close(self):
        self.closed = True
        for t in list(self._watch_tasks):
            t.cancel()
        if self.channel is not None:
            await self.channel.close()

    # -- key / value translation --------------------------------------------------------------
    def _k(self, key: str) -> bytes:
        return (self.namespace + key).encode("utf-8", "surrogateescape")

    def _unk(self, key: bytes) -> str:
        k = key.decode("utf-8", "surrogateescape")
        return k[len(self.namespace):] if self.namespace and k.startswith(self.namespace) else k

    @staticmethod
    def _inject(v: bytes, tok: bytes) -> bytes:
        """The stored form of a PUT_INJECT value: the token's offsets, then the value without it."""
        parts = v.split(tok) if tok else [v]
        offs, pos = [], 0
        for part in parts[:-1]:
            pos += len(part)
            offs.append(pos)
        if len(offs) > 0xFFFF:
            raise Etcd3Error("too many resourceVersion tokens in one value")
        return INJECT_MAGIC + len(offs).to_bytes(2, "big") + b"".join(o.to_bytes(4, "big") for o in offs) + b"".join(parts)

    @staticmethod
    def _value(v: bytes, mod_rev: int) -> bytes:
        if not v.startswith(INJECT_MAGIC):
            return v
        n = int.from_bytes(v[4:6], "big")
        body = v[6 + 4 * n:]
        if not n:
            return body
        rv = str(mod_rev).encode()
        out, last = [], 0
        for i in range(n):
            o = int.from_bytes(v[6 + 4 * i:10 + 4 * i], "big")
            out.append(body[last:o])
            out.append(rv)
            last = o
        out.append(body[last:])
        return b"".join(out)

    def _kv(self, pkv, value=None, mod_rev=None) -> KV:
        mr = mod_rev if mod_rev is not None else pkv.mod_revision
        v = pkv.value if value is None else value
        return KV(self._unk(pkv.key), self._value(v, mr), pkv.create_revision, mr, pkv.version)

    # -- reads --------------------------------------------------------------------------------
    async def get(self, key):
        r = await self._Range(M["RangeRequest"](key=self._k(key)))
        return self._kv(r.kvs[0]) if r.kvs else None

    async def revision(self):
        r = await self._Range(M["RangeRequest"](key=self._k("/"), count_only=True))
        return r.header.revision

    async def range(self, prefix, limit=0, start_after=None, revision=0):
        """(kvs, more, revision) of the keys with `prefix` (strictly after `start_after`). An
        unlimited range is read in pages pinned to the first page's revision (one consistent
        snapshot, like the reference's paged LIST)."""
        end = prefix_end(self._k(prefix)) if prefix else b"\x00"
        start = self._k(start_after) + b"\x00" if start_after else (self._k(prefix) if prefix else self._k(""))
        if not self.namespace and not prefix and not start_after:
            start = b"\x00"
        out, rev = [], revision
        while True:
            want = limit - len(out) if limit else _PAGE
            try:
                r = await self._Range(M["RangeRequest"](key=start, range_end=end, limit=want, revision=rev))
            except grpc.aio.AioRpcError as e:
                if "compacted" in (e.details() or ""):
                    raise CompactedError(rev) from None
                raise
            rev = rev or r.header.revision
            out += [self._kv(kv) for kv in r.kvs]
            if not r.more or not r.kvs:
                return out, False, rev
            if limit and len(out) >= limit:
                return out, True, rev
            start = r.kvs[-1].key + b"\x00"

    # -- writes -------------------------------------------------------------------------------
    def _compare(self, kind, key, arg, val):
        k = self._k(key)
        if kind == wire.CMP_MOD_REV:
            return M["Compare"](key=k, target=T_MOD, result=EQUAL, mod_revision=arg)
        if kind == wire.CMP_EXISTS:
            return M["Compare"](key=k, target=T_VERSION, result=GREATER, version=0)
        if kind == wire.CMP_ABSENT:
            return M["Compare"](key=k, target=T_VERSION, result=EQUAL, version=0)
        if kind == wire.CMP_VALUE:
            return M["Compare"](key=k, target=T_VALUE, result=EQUAL, value=val or b"")
        raise Etcd3Error(f"unknown compare kind {kind}")

    def _op(self, op):
        kind, key, val = op[0], op[1], op[2]
        if kind == wire.OP_PUT:
            return M["RequestOp"](request_put=M["PutRequest"](key=self._k(key), value=val or b""))
        if kind == wire.OP_PUT_INJECT:
            return M["RequestOp"](request_put=M["PutRequest"](key=self._k(key), value=self._inject(val or b"", op[3])))
        if kind in (wire.OP_DELETE, wire.OP_DELETE_TOMBSTONE):
            return M["RequestOp"](request_delete_range=M["DeleteRangeRequest"](key=self._k(key)))
        raise Etcd3Error(f"unknown op kind {kind}")

    @staticmethod
    def _holds(kind, arg, val, kv):
        if kind == wire.CMP_MOD_REV:
            return (kv.mod_revision if kv is not None else 0) == arg
        if kind == wire.CMP_EXISTS:
            return kv is not None
        if kind == wire.CMP_ABSENT:
            return kv is None
        return kv is not None and kv.value == (val or b"")

    async def txn(self, cmps, ops, on_ok=None) -> TxnResult:
        keys = list(dict.fromkeys(c[1] for c in cmps))
        req = M["TxnRequest"](compare=[self._compare(*c) for c in cmps], success=[self._op(o) for o in ops],
                              failure=[M["RequestOp"](request_range=M["RangeRequest"](key=self._k(k))) for k in keys])
        r = await self._Txn(req)
        rev = r.header.revision
        if r.succeeded:
            if on_ok is not None:
                on_ok(rev)
            return TxnResult(True, rev)
        seen = {}
        for k, resp in zip(keys, r.responses):
            kvs = resp.response_range.kvs
            seen[k] = kvs[0] if kvs else None
        for i, (kind, key, arg, val) in enumerate(cmps):
            cur = seen.get(key)
            if not self._holds(kind, arg, val, cur):
                return TxnResult(False, rev, i, self._kv(cur) if cur is not None else None)
        # every compare holds on the failure branch's read: the key changed back in between
        return TxnResult(False, rev, 0, self._kv(seen[keys[0]]) if keys and seen.get(keys[0]) else None)

    async def compact(self, rev):
        await self._Compact(M["CompactionRequest"](revision=rev))

    # -- watch --------------------------------------------------------------------------------
    async def watch(self, prefix, from_rev, callback, exclude=()):
        """callback(type, kv) for every event after `from_rev` (0 = from now), in revision
        order; callback(None, None) when the stream ends. Returns the revision at creation.
        Raises CompactedError when `from_rev` is older than the retained history."""
        queue: asyncio.Queue = asyncio.Queue()
        end = prefix_end(self._k(prefix)) if prefix else b"\x00"
        start = self._k(prefix) if (prefix or self.namespace) else b"\x00"
        create = M["WatchRequest"](create_request=M["WatchCreateRequest"](
            key=start, range_end=end, start_revision=from_rev + 1 if from_rev else 0, prev_kv=True))
        queue.put_nowait(create)
        excl = tuple(self._k(x) for x in exclude)

        async def requests():
            while True:
                m = await queue.get()
                if m is None:
                    return
                yield m
        call = self._Watch(requests())
        it = call.__aiter__()
        try:
            first = await it.__anext__()
            if first.canceled or first.compact_revision:
                raise CompactedError(from_rev)
            if not first.created:
                raise Etcd3Error("etcd watch was not created")
            created_rev = first.header.revision
            # etcd may send the compaction cancel right after `created`
        except (grpc.aio.AioRpcError, StopAsyncIteration) as e:
            call.cancel()
            raise Etcd3Error(f"etcd watch failed: {e}") from None

        def deliver(resp):
            if resp.canceled:
                return False
            for ev in resp.events:
                key = ev.kv.key
                if excl and key.startswith(excl):
                    callback(wire.PROGRESS, ev.kv.mod_revision)
                    continue
                if ev.type == 1:      # DELETE: the deleted object is prev_kv
                    pv = ev.prev_kv if ev.HasField("prev_kv") else None
                    kv = self._kv(pv if pv is not None else ev.kv, mod_rev=ev.kv.mod_revision)
                    kv.version = 0
                    callback(1, kv)
                else:
                    callback(0, self._kv(ev.kv))
            return True

        async def pump():
            try:
                async for resp in it:
                    if resp.compact_revision and resp.canceled:
                        log.warning("etcd watch on %s compacted at %d", prefix, resp.compact_revision)
                        break
                    if not deliver(resp):
                        break
            except asyncio.CancelledError:
                raise
            except grpc.aio.AioRpcError as e:
                if not self.closed:
                    log.error("etcd watch on %s ended: %s %s", prefix, e.code().name, e.details())
            finally:
                queue.put_nowait(None)
                try:
                    callback(None, None)
                except Exception:  # noqa: BLE001 - the stream is over either way
                    pass
        t = asyncio.ensure_future(pump())
        self._watch_tasks.add(t)
        t.add_done_callback(self._watch_tasks.discard)
        return created_rev


async def connect_store(address, tls=None):
    """The store client for an `--etcd-servers` value: an etcd v3 endpoint (http/https URL) or
    the native store (`unix://PATH`, `tcp://HOST:PORT`)."""
    if is_etcd3_address(address):
        return await Etcd3Store(address, tls=tls).connect()
    from .remote import RemoteStore
    return await RemoteStore(address).connect()
