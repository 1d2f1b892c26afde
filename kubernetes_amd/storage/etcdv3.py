"""etcd v3 gRPC API over the native store (kamd-etcd): etcdctl / etcd client libraries can read,
write and watch the cluster state the API server keeps there.

Parity: the etcd v3 API the reference API server is a client of (`staging/src/k8s.io/apiserver/
pkg/storage/etcd3`, wire schema `vendor/github.com/coreos/etcd/etcdserver/etcdserverpb/rpc.proto`
+ `mvcc/mvccpb/kv.proto` — only field numbers are taken from there):

  * KV: Range (single key, `[key, range_end)`, `range_end == "\\0"` = from key to the end;
    limit / count_only / keys_only / sort), Put (prev_kv, lease), DeleteRange (prev_kv), Txn
    (Compare on VERSION / CREATE / MOD / VALUE with EQUAL / GREATER / LESS / NOT_EQUAL; Put /
    DeleteRange / Range ops), Compact;
  * Watch: bidirectional stream, several watches per stream, start_revision replay, NOPUT /
    NODELETE filters, `canceled` + `compact_revision` for a compacted start;
  * Lease: Grant / Revoke / KeepAlive / TimeToLive — leases live in this gateway (not in the
    store): expiry deletes the attached keys;
  * Maintenance.Status (revision, db size, version).

Txn atomicity: the compares are evaluated on a read of their keys, and the chosen branch commits
in ONE store transaction guarded by the mod revisions that read saw (absent keys guarded as
absent); a concurrent change fails the guard and the Txn is re-evaluated — the same outcome as
etcd's serialized Txn for the keys it compares. Range at a past `revision` is served by the
store (its retained history undone from the current state): "required revision has been
compacted" below it, "required revision is a future revision" above the current one. Watch
replays events after `start_revision - 1` (0 = from now); `prev_kv` is filled for DELETE events
(the deleted key's last value, as clientv3 users such as the API server's watcher expect).
"""
from __future__ import annotations

import asyncio
import itertools
import logging
import time

import grpc

from ..utils.protodesc import build
from . import wire
from .mvcc import CompactedError, DELETE, PUT
from .remote import RemoteStore

log = logging.getLogger("etcdv3")

PKG = "etcdserverpb"
_KV = [("key", 1, "bytes", "opt", None), ("create_revision", 2, "int64", "opt", None),
       ("mod_revision", 3, "int64", "opt", None), ("version", 4, "int64", "opt", None),
       ("value", 5, "bytes", "opt", None), ("lease", 6, "int64", "opt", None)]
_HDR = ("header", 1, "message", "opt", "ResponseHeader")
SCHEMA = {
    "ResponseHeader": [("cluster_id", 1, "uint64", "opt", None), ("member_id", 2, "uint64", "opt", None),
                       ("revision", 3, "int64", "opt", None), ("raft_term", 4, "uint64", "opt", None)],
    "KeyValue": _KV,
    "Event": [("type", 1, "int32", "opt", None), ("kv", 2, "message", "opt", "KeyValue"),
              ("prev_kv", 3, "message", "opt", "KeyValue")],
    "RangeRequest": [("key", 1, "bytes", "opt", None), ("range_end", 2, "bytes", "opt", None),
                     ("limit", 3, "int64", "opt", None), ("revision", 4, "int64", "opt", None),
                     ("sort_order", 5, "int32", "opt", None), ("sort_target", 6, "int32", "opt", None),
                     ("serializable", 7, "bool", "opt", None), ("keys_only", 8, "bool", "opt", None),
                     ("count_only", 9, "bool", "opt", None), ("min_mod_revision", 10, "int64", "opt", None),
                     ("max_mod_revision", 11, "int64", "opt", None),
                     ("min_create_revision", 12, "int64", "opt", None),
                     ("max_create_revision", 13, "int64", "opt", None)],
    "RangeResponse": [_HDR, ("kvs", 2, "message", "rep", "KeyValue"), ("more", 3, "bool", "opt", None),
                      ("count", 4, "int64", "opt", None)],
    "PutRequest": [("key", 1, "bytes", "opt", None), ("value", 2, "bytes", "opt", None),
                   ("lease", 3, "int64", "opt", None), ("prev_kv", 4, "bool", "opt", None)],
    "PutResponse": [_HDR, ("prev_kv", 2, "message", "opt", "KeyValue")],
    "DeleteRangeRequest": [("key", 1, "bytes", "opt", None), ("range_end", 2, "bytes", "opt", None),
                           ("prev_kv", 3, "bool", "opt", None)],
    "DeleteRangeResponse": [_HDR, ("deleted", 2, "int64", "opt", None), ("prev_kvs", 3, "message", "rep", "KeyValue")],
    "RequestOp": [("request_range", 1, "message", "oneof:request", "RangeRequest"),
                  ("request_put", 2, "message", "oneof:request", "PutRequest"),
                  ("request_delete_range", 3, "message", "oneof:request", "DeleteRangeRequest")],
    "ResponseOp": [("response_range", 1, "message", "oneof:response", "RangeResponse"),
                   ("response_put", 2, "message", "oneof:response", "PutResponse"),
                   ("response_delete_range", 3, "message", "oneof:response", "DeleteRangeResponse")],
    "Compare": [("result", 1, "int32", "opt", None), ("target", 2, "int32", "opt", None), ("key", 3, "bytes", "opt", None),
                ("version", 4, "int64", "oneof:target_union", None),
                ("create_revision", 5, "int64", "oneof:target_union", None),
                ("mod_revision", 6, "int64", "oneof:target_union", None),
                ("value", 7, "bytes", "oneof:target_union", None)],
    "TxnRequest": [("compare", 1, "message", "rep", "Compare"), ("success", 2, "message", "rep", "RequestOp"),
                   ("failure", 3, "message", "rep", "RequestOp")],
    "TxnResponse": [_HDR, ("succeeded", 2, "bool", "opt", None), ("responses", 3, "message", "rep", "ResponseOp")],
    "CompactionRequest": [("revision", 1, "int64", "opt", None), ("physical", 2, "bool", "opt", None)],
    "CompactionResponse": [_HDR],
    "WatchCreateRequest": [("key", 1, "bytes", "opt", None), ("range_end", 2, "bytes", "opt", None),
                           ("start_revision", 3, "int64", "opt", None), ("progress_notify", 4, "bool", "opt", None),
                           ("filters", 5, "int32", "rep", None), ("prev_kv", 6, "bool", "opt", None)],
    "WatchCancelRequest": [("watch_id", 1, "int64", "opt", None)],
    "WatchRequest": [("create_request", 1, "message", "oneof:request_union", "WatchCreateRequest"),
                     ("cancel_request", 2, "message", "oneof:request_union", "WatchCancelRequest")],
    "WatchResponse": [_HDR, ("watch_id", 2, "int64", "opt", None), ("created", 3, "bool", "opt", None),
                      ("canceled", 4, "bool", "opt", None), ("compact_revision", 5, "int64", "opt", None),
                      ("events", 11, "message", "rep", "Event")],
    "LeaseGrantRequest": [("TTL", 1, "int64", "opt", None), ("ID", 2, "int64", "opt", None)],
    "LeaseGrantResponse": [_HDR, ("ID", 2, "int64", "opt", None), ("TTL", 3, "int64", "opt", None),
                           ("error", 4, "string", "opt", None)],
    "LeaseRevokeRequest": [("ID", 1, "int64", "opt", None)],
    "LeaseRevokeResponse": [_HDR],
    "LeaseKeepAliveRequest": [("ID", 1, "int64", "opt", None)],
    "LeaseKeepAliveResponse": [_HDR, ("ID", 2, "int64", "opt", None), ("TTL", 3, "int64", "opt", None)],
    "LeaseTimeToLiveRequest": [("ID", 1, "int64", "opt", None), ("keys", 2, "bool", "opt", None)],
    "LeaseTimeToLiveResponse": [_HDR, ("ID", 2, "int64", "opt", None), ("TTL", 3, "int64", "opt", None),
                                ("grantedTTL", 4, "int64", "opt", None), ("keys", 5, "bytes", "rep", None)],
    "StatusRequest": [],
    "StatusResponse": [_HDR, ("version", 2, "string", "opt", None), ("dbSize", 3, "int64", "opt", None),
                       ("leader", 4, "uint64", "opt", None), ("raftIndex", 5, "uint64", "opt", None),
                       ("raftTerm", 6, "uint64", "opt", None)],
}
M = build(PKG, "kamd_etcd_rpc.proto", SCHEMA)

# service -> {method: (request, response, kind)} ; kind: unary | stream (bidi)
SERVICES = {
    "KV": {"Range": ("RangeRequest", "RangeResponse", "unary"), "Put": ("PutRequest", "PutResponse", "unary"),
           "DeleteRange": ("DeleteRangeRequest", "DeleteRangeResponse", "unary"),
           "Txn": ("TxnRequest", "TxnResponse", "unary"), "Compact": ("CompactionRequest", "CompactionResponse", "unary")},
    "Watch": {"Watch": ("WatchRequest", "WatchResponse", "stream")},
    "Lease": {"LeaseGrant": ("LeaseGrantRequest", "LeaseGrantResponse", "unary"),
              "LeaseRevoke": ("LeaseRevokeRequest", "LeaseRevokeResponse", "unary"),
              "LeaseKeepAlive": ("LeaseKeepAliveRequest", "LeaseKeepAliveResponse", "stream"),
              "LeaseTimeToLive": ("LeaseTimeToLiveRequest", "LeaseTimeToLiveResponse", "unary")},
    "Maintenance": {"Status": ("StatusRequest", "StatusResponse", "unary")},
}
EQUAL, GREATER, LESS, NOT_EQUAL = 0, 1, 2, 3
T_VERSION, T_CREATE, T_MOD, T_VALUE = 0, 1, 2, 3
NOPUT, NODELETE = 0, 1
CLUSTER_ID, MEMBER_ID = 0x6B616D64, 0x1
VERSION = "3.1.11-kamd"


def prefix_end(key: bytes) -> bytes:
    """The range_end that selects every key with prefix `key` (clientv3.GetPrefixRangeEnd)."""
    k = bytearray(key)
    for i in range(len(k) - 1, -1, -1):
        if k[i] < 0xFF:
            k[i] += 1
            return bytes(k[:i + 1])
    return b"\x00"


def _common_prefix(a: bytes, b: bytes) -> bytes:
    n = 0
    while n < min(len(a), len(b)) and a[n] == b[n]:
        n += 1
    return a[:n]


def _in_range(key: bytes, start: bytes, end: bytes) -> bool:
    if not end:
        return key == start
    if end == b"\x00":
        return key >= start
    return start <= key < end


class EtcdV3Gateway:
    def __init__(self, store_address: str):
        self.address = store_address
        self.store: RemoteStore | None = None
        self.server = None
        self.port = None
        self.leases: dict[int, dict] = {}          # id -> {"ttl", "granted", "expires", "keys": set}
        self._lease_ids = itertools.count(int(time.time()) << 16)
        self._reaper = None
        self.compacted = 0

    # -- lifecycle --------------------------------------------------------------------------------
    async def start(self, listen="127.0.0.1:0"):
        self.store = await RemoteStore(self.address).connect()
        self.server = grpc.aio.server()
        for svc, methods in SERVICES.items():
            handlers = {}
            for name, (req, resp, kind) in methods.items():
                fn = getattr(self, name)
                if kind == "stream":
                    handlers[name] = grpc.stream_stream_rpc_method_handler(
                        fn, request_deserializer=M[req].FromString, response_serializer=M[resp].SerializeToString)
                else:
                    handlers[name] = grpc.unary_unary_rpc_method_handler(
                        fn, request_deserializer=M[req].FromString, response_serializer=M[resp].SerializeToString)
            self.server.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(f"{PKG}.{svc}", handlers),))
        self.port = self.server.add_insecure_port(listen)
        await self.server.start()
        self._reaper = asyncio.ensure_future(self._expire_leases())
        return self

    async def stop(self):
        if self._reaper:
            self._reaper.cancel()
        if self.server is not None:
            await self.server.stop(0.2)
        if self.store is not None:
            await self.store.close()

    async def _header(self, rev=None):
        return M["ResponseHeader"](cluster_id=CLUSTER_ID, member_id=MEMBER_ID,
                                   revision=rev if rev is not None else await self.store.revision(), raft_term=1)

    def _kv(self, kv, keys_only=False):
        lease = next((lid for lid, l in self.leases.items() if kv.key in l["keys"]), 0)
        return M["KeyValue"](key=kv.key.encode(), create_revision=kv.create_rev, mod_revision=kv.mod_rev,
                             version=kv.version, value=b"" if keys_only else kv.value, lease=lease)

    # -- reads ------------------------------------------------------------------------------------
    async def _range_kvs(self, key: bytes, end: bytes, revision=0):
        if not end and not revision:
            kv = await self.store.get(key.decode())
            return [kv] if kv is not None else []
        if not end:
            kvs, _more, _rev = await self.store.range(key.decode(errors="surrogateescape"), revision=revision)
            return [kv for kv in kvs if kv.key.encode() == key]
        prefix = key if end == b"\x00" else _common_prefix(key, end)
        kvs, _more, _rev = await self.store.range(prefix.decode(errors="surrogateescape"), revision=revision)
        return [kv for kv in kvs if _in_range(kv.key.encode(), key, end)]

    async def Range(self, req, ctx):
        rev = await self.store.revision()
        at = 0
        if req.revision and req.revision < rev:
            at = req.revision
        elif req.revision > rev:
            await ctx.abort(grpc.StatusCode.OUT_OF_RANGE, "etcdserver: mvcc: required revision is a future revision")
        try:
            kvs = await self._range_kvs(req.key, req.range_end, at)
        except CompactedError:
            await ctx.abort(grpc.StatusCode.OUT_OF_RANGE, "etcdserver: mvcc: required revision has been compacted")
        kvs = [kv for kv in kvs if (not req.min_mod_revision or kv.mod_rev >= req.min_mod_revision)
               and (not req.max_mod_revision or kv.mod_rev <= req.max_mod_revision)
               and (not req.min_create_revision or kv.create_rev >= req.min_create_revision)
               and (not req.max_create_revision or kv.create_rev <= req.max_create_revision)]
        if req.sort_order:
            key = {0: lambda k: k.key, 1: lambda k: k.version, 2: lambda k: k.create_rev,
                   3: lambda k: k.mod_rev, 4: lambda k: k.value}[req.sort_target]
            kvs.sort(key=key, reverse=req.sort_order == 2)
        count = len(kvs)
        more = bool(req.limit) and count > req.limit
        if req.limit:
            kvs = kvs[:req.limit]
        return M["RangeResponse"](header=await self._header(at or None), count=count, more=more,
                                  kvs=[] if req.count_only else [self._kv(kv, req.keys_only) for kv in kvs])

    # -- writes -------------------------------------------------------------------------------------
    async def Put(self, req, ctx):
        prev = await self.store.get(req.key.decode()) if req.prev_kv else None
        r = await self.store.txn([], [(wire.OP_PUT, req.key.decode(), req.value)])
        self._attach(req.key.decode(), req.lease)
        resp = M["PutResponse"](header=await self._header(r.rev))
        if prev is not None:
            resp.prev_kv.CopyFrom(self._kv(prev))
        return resp

    def _attach(self, key, lease):
        for l in self.leases.values():
            l["keys"].discard(key)
        if lease and lease in self.leases:
            self.leases[lease]["keys"].add(key)

    async def DeleteRange(self, req, ctx):
        kvs = await self._range_kvs(req.key, req.range_end)
        rev = await self.store.revision()
        if kvs:
            r = await self.store.txn([], [(wire.OP_DELETE, kv.key, b"") for kv in kvs])
            rev = r.rev
            for kv in kvs:
                self._attach(kv.key, 0)
        return M["DeleteRangeResponse"](header=await self._header(rev), deleted=len(kvs),
                                        prev_kvs=[self._kv(kv) for kv in kvs] if req.prev_kv else [])

    @staticmethod
    def _compare(c, kv) -> bool:
        which = c.WhichOneof("target_union")
        if c.target == T_VALUE:
            have, want = (kv.value if kv else None), c.value
            if have is None:
                return False
        else:
            have = 0 if kv is None else {T_VERSION: kv.version, T_CREATE: kv.create_rev, T_MOD: kv.mod_rev}[c.target]
            want = getattr(c, which) if which else 0
        return {EQUAL: have == want, GREATER: have > want, LESS: have < want, NOT_EQUAL: have != want}[c.result]

    async def Txn(self, req, ctx):
        for _ in range(16):
            keys = sorted({c.key for c in req.compare})
            seen = {k: await self.store.get(k.decode()) for k in keys}
            ok = all(self._compare(c, seen[c.key]) for c in req.compare)
            branch = req.success if ok else req.failure
            guards = [(wire.CMP_MOD_REV, k.decode(), kv.mod_rev, b"") if kv is not None else
                      (wire.CMP_ABSENT, k.decode(), 0, b"") for k, kv in seen.items()]
            ops, deleted, puts, pending = [], {}, [], []
            for op in branch:
                kind = op.WhichOneof("request")
                if kind == "request_put":
                    ops.append((wire.OP_PUT, op.request_put.key.decode(), op.request_put.value))
                    puts.append(op.request_put)
                elif kind == "request_delete_range":
                    d = op.request_delete_range
                    kvs = await self._range_kvs(d.key, d.range_end)
                    deleted[id(op)] = kvs
                    for kv in kvs:
                        guards.append((wire.CMP_MOD_REV, kv.key, kv.mod_rev, b""))
                        ops.append((wire.OP_DELETE, kv.key, b""))
                pending.append((kind, op))
            if ops:
                r = await self.store.txn(guards, ops)
                if not r.ok:
                    continue                      # a compared key changed under us: re-evaluate
                rev = r.rev
            else:
                rev = await self.store.revision()
            for p in puts:
                self._attach(p.key.decode(), p.lease)
            hdr = await self._header(rev)
            responses = []
            for kind, op in pending:
                if kind == "request_put":
                    responses.append(M["ResponseOp"](response_put=M["PutResponse"](header=hdr)))
                elif kind == "request_delete_range":
                    kvs = deleted[id(op)]
                    responses.append(M["ResponseOp"](response_delete_range=M["DeleteRangeResponse"](
                        header=hdr, deleted=len(kvs), prev_kvs=[self._kv(kv) for kv in kvs]
                        if op.request_delete_range.prev_kv else [])))
                else:
                    responses.append(M["ResponseOp"](response_range=await self.Range(op.request_range, ctx)))
            return M["TxnResponse"](header=hdr, succeeded=ok, responses=responses)
        await ctx.abort(grpc.StatusCode.ABORTED, "etcdserver: too much contention on the compared keys")

    async def Compact(self, req, ctx):
        await self.store.compact(req.revision)
        self.compacted = max(self.compacted, req.revision)
        return M["CompactionResponse"](header=await self._header())

    # -- watch --------------------------------------------------------------------------------------
    async def Watch(self, request_iterator, ctx):
        """One dedicated store connection per Watch stream; each create_request is a store
        watch on the key range's common prefix, filtered to the range."""
        out: asyncio.Queue = asyncio.Queue()
        conn = await RemoteStore(self.address).connect()
        active: dict[int, tuple] = {}
        ids = itertools.count(0)

        async def reader():
            try:
                async for wr in request_iterator:
                    which = wr.WhichOneof("request_union")
                    if which == "create_request":
                        await create(wr.create_request)
                    elif which == "cancel_request":
                        wid = wr.cancel_request.watch_id
                        active.pop(wid, None)
                        out.put_nowait(M["WatchResponse"](header=await self._header(), watch_id=wid, canceled=True))
            finally:
                out.put_nowait(None)

        async def create(cr):
            wid = next(ids)
            start, end = cr.key, cr.range_end
            prefix = start if end == b"\x00" else (_common_prefix(start, end) if end else start)
            filters = set(cr.filters)
            active[wid] = (start, end)
            # replayed events can arrive before the store's watch reply is processed: hold them
            # until `created` is out (etcd sends `created` first)
            held = []

            def cb(t, kv):
                if t is None or wid not in active or t == wire.PROGRESS:
                    return
                if not _in_range(kv.key.encode(), start, end):
                    return
                etype = DELETE if t == DELETE else PUT
                if (etype == PUT and NOPUT in filters) or (etype == DELETE and NODELETE in filters):
                    return
                ev = M["Event"](type=etype, kv=self._kv(kv))
                if etype == DELETE:
                    if cr.prev_kv:
                        # the store's delete event carries the key's last value
                        ev.prev_kv.CopyFrom(self._kv(kv))
                        ev.prev_kv.version = max(1, kv.version)
                    ev.kv.value = b""
                    ev.kv.version = 0
                    ev.kv.create_revision = 0
                resp = M["WatchResponse"](header=M["ResponseHeader"](
                    cluster_id=CLUSTER_ID, member_id=MEMBER_ID, revision=kv.mod_rev, raft_term=1),
                    watch_id=wid, events=[ev])
                if held is not None:
                    held.append(resp)
                else:
                    out.put_nowait(resp)
            try:
                rev = await conn.watch(prefix.decode(errors="surrogateescape"),
                                       max(0, cr.start_revision - 1) if cr.start_revision else 0, cb)
                out.put_nowait(M["WatchResponse"](header=await self._header(rev), watch_id=wid, created=True))
                pending, held = held, None
                for resp in pending:
                    out.put_nowait(resp)
            except CompactedError:
                active.pop(wid, None)
                # created and canceled at once, with the compaction point the client must resume
                # from (the store's compaction revision when this gateway performed it; at least
                # the requested start)
                out.put_nowait(M["WatchResponse"](header=await self._header(), watch_id=wid, created=True,
                                                  canceled=True,
                                                  compact_revision=max(self.compacted, cr.start_revision)))
        task = asyncio.ensure_future(reader())
        try:
            while True:
                m = await out.get()
                if m is None:
                    return
                yield m
        finally:
            task.cancel()
            await conn.close()

    # -- leases -------------------------------------------------------------------------------------
    async def LeaseGrant(self, req, ctx):
        lid = req.ID or next(self._lease_ids)
        if lid in self.leases:
            return M["LeaseGrantResponse"](header=await self._header(), ID=lid, error="etcdserver: lease already exists")
        now = time.monotonic()
        self.leases[lid] = {"ttl": req.TTL, "granted": req.TTL, "expires": now + req.TTL, "keys": set()}
        return M["LeaseGrantResponse"](header=await self._header(), ID=lid, TTL=req.TTL)

    async def _revoke(self, lid):
        l = self.leases.pop(lid, None)
        if l and l["keys"]:
            await self.store.txn([], [(wire.OP_DELETE, k, b"") for k in sorted(l["keys"])])

    async def LeaseRevoke(self, req, ctx):
        if req.ID not in self.leases:
            await ctx.abort(grpc.StatusCode.NOT_FOUND, "etcdserver: requested lease not found")
        await self._revoke(req.ID)
        return M["LeaseRevokeResponse"](header=await self._header())

    async def LeaseKeepAlive(self, request_iterator, ctx):
        async for r in request_iterator:
            l = self.leases.get(r.ID)
            if l is None:
                yield M["LeaseKeepAliveResponse"](header=await self._header(), ID=r.ID, TTL=0)
                continue
            l["expires"] = time.monotonic() + l["granted"]
            yield M["LeaseKeepAliveResponse"](header=await self._header(), ID=r.ID, TTL=l["granted"])

    async def LeaseTimeToLive(self, req, ctx):
        l = self.leases.get(req.ID)
        if l is None:
            return M["LeaseTimeToLiveResponse"](header=await self._header(), ID=req.ID, TTL=-1)
        return M["LeaseTimeToLiveResponse"](header=await self._header(), ID=req.ID,
                                            TTL=max(0, int(l["expires"] - time.monotonic())), grantedTTL=l["granted"],
                                            keys=[k.encode() for k in sorted(l["keys"])] if req.keys else [])

    async def _expire_leases(self):
        while True:
            await asyncio.sleep(0.2)
            now = time.monotonic()
            for lid in [lid for lid, l in self.leases.items() if l["expires"] <= now]:
                try:
                    await self._revoke(lid)
                except Exception:  # noqa: BLE001 - retried on the next tick
                    log.exception("lease %x expiry failed", lid)

    # -- maintenance -------------------------------------------------------------------------------
    async def Status(self, req, ctx):
        rev = await self.store.revision()
        kvs, _m, _r = await self.store.range("")
        size = sum(len(kv.key) + len(kv.value) for kv in kvs)
        return M["StatusResponse"](header=await self._header(rev), version=VERSION, dbSize=size, leader=MEMBER_ID,
                                   raftIndex=rev, raftTerm=1)


class EtcdV3Client:
    """Minimal clientv3 over grpc.aio (tests, `kamd` tools)."""

    def __init__(self, target: str):
        self.channel = grpc.aio.insecure_channel(target)
        for svc, methods in SERVICES.items():
            for name, (req, resp, kind) in methods.items():
                path = f"/{PKG}.{svc}/{name}"
                mk = self.channel.stream_stream if kind == "stream" else self.channel.unary_unary
                setattr(self, name, mk(path, request_serializer=M[req].SerializeToString,
                                       response_deserializer=M[resp].FromString))

    async def close(self):
        await self.channel.close()
