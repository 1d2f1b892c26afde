"""Watch cache + watcher fan-out (one `ResourceCache` per resource).

Parity: `staging/src/k8s.io/apiserver/pkg/storage/cacher.go:141-667` (`Cacher`,
`dispatchEvent`, indexed watchers by `spec.nodeName` for pods) and `watch_cache.go`
(sliding window of recent events for resuming watches, 410 Gone when too old).

Design notes (MI355X host side, Python): every object is JSON-encoded exactly once, at
write time; that byte string is what the KV store holds, what GET returns, what LIST joins
and what every watch event embeds — so a write with W interested watchers costs one
encode + W socket writes, not W encodes.
"""
from __future__ import annotations

import logging
from collections import deque

from ..api import codec
from ..api.labels import parse as parse_labels, parse_field_selector
from ..api.sharding import shard_matches

log = logging.getLogger("cacher")

ADDED, MODIFIED, DELETED, BOOKMARK, ERROR = "ADDED", "MODIFIED", "DELETED", "BOOKMARK", "ERROR"


class Entry:
    """One cached object version. `obj` may be decoded lazily: an API server worker that only
    relays another worker's write needs the raw bytes (GET/LIST/watch payload) and the index
    fields/labels (watch + list filtering) — not the decoded object. `pbv`: the stored protobuf
    envelope when there is one (without resourceVersion, as etcd3 stores it); `pb_envelope()`
    is what protobuf watchers are sent."""
    __slots__ = ("_obj", "_raw", "rev", "fields", "labels", "pbv", "_pb")

    def __init__(self, obj, raw, rev, fields, labels=None, pbv=None):
        # raw may be None when pbv is set: the JSON form is then made on first use (a write
        # answered to a protobuf client never needs it)
        self._obj, self._raw, self.rev, self.fields = obj, raw, rev, fields
        self.labels = labels if obj is None else ((obj.get("metadata") or {}).get("labels") or {})
        self.pbv = pbv
        self._pb = None

    @property
    def raw(self):
        r = self._raw
        if r is None:
            from ..api import protobuf as pb
            r = self._raw = pb.to_json(self.pbv, self.rev) if self.pbv is not None else codec.dumpb(self._obj)
        return r

    def pb_envelope(self):
        """The object as a `k8s\\x00` protobuf envelope with its resourceVersion, or its JSON bytes
        for kinds outside the protobuf schema (a protobuf watch embeds those as-is; clients tell
        them apart by the magic)."""
        b = self._pb
        if b is None:
            from ..api import protobuf as pb
            if self.pbv is not None:
                b = pb.envelope_with_rv(self.pbv, str(self.rev))
            if b is None:
                o = self.obj
                b = pb.encode_object(o) if pb.supported(o.get("kind", ""), o.get("apiVersion") or "v1") else self.raw
            self._pb = b
        return b

    @property
    def obj(self):
        o = self._obj
        if o is None:
            if self._raw is None and self.pbv is not None:
                from ..api import protobuf as pb
                o = pb.decode_storage(self.pbv)
                o.setdefault("metadata", {})["resourceVersion"] = str(self.rev)
            else:
                o = codec.loads(self.raw)
            self._obj = o
        return o

    @property
    def sort_key(self):
        f = self.fields
        return f.get("metadata.namespace", "") + "/" + f.get("metadata.name", "")


UNINITIALIZED = "metadata.uninitialized"


class GoneError(Exception):
    pass


def pod_fields(obj):
    m = obj.get("metadata") or {}
    s = obj.get("spec") or {}
    st = obj.get("status") or {}
    return {
        "metadata.name": m.get("name", ""),
        "metadata.namespace": m.get("namespace", ""),
        "spec.nodeName": s.get("nodeName", ""),
        "spec.restartPolicy": s.get("restartPolicy", ""),
        "spec.schedulerName": s.get("schedulerName", ""),
        "status.phase": st.get("phase", ""),
        "status.podIP": st.get("podIP", ""),
    }


def node_fields(obj):
    m = obj.get("metadata") or {}
    return {"metadata.name": m.get("name", ""),
            "spec.unschedulable": str(bool((obj.get("spec") or {}).get("unschedulable", False))).lower()}


def generic_fields(obj):
    m = obj.get("metadata") or {}
    f = {"metadata.name": m.get("name", ""), "metadata.namespace": m.get("namespace", "")}
    if obj.get("kind") == "Event":
        io = obj.get("involvedObject") or {}
        f.update({"involvedObject.kind": io.get("kind", ""), "involvedObject.name": io.get("name", ""),
                  "involvedObject.namespace": io.get("namespace", ""), "involvedObject.uid": io.get("uid", ""),
                  "reason": obj.get("reason", ""), "type": obj.get("type", "")})
    if obj.get("kind") == "Secret":
        f["type"] = obj.get("type", "")
    if obj.get("kind") == "Namespace":
        f["status.phase"] = (obj.get("status") or {}).get("phase", "")
    return f


FIELD_FUNCS = {"pods": pod_fields, "nodes": node_fields}


class Watcher:
    __slots__ = ("writer", "namespace", "label_sel", "field_sel", "closed", "index_value", "cache", "bookmarks",
                 "_pending", "_loop", "min_rev", "shard", "pb")

    def __init__(self, cache, writer, namespace, label_sel, field_sel, index_value):
        self.cache = cache
        # events at or below this revision are already reflected in what the client has (its
        # list came from a worker that was further ahead than this one): never re-send them
        self.min_rev = 0
        self.writer = writer
        self.namespace = namespace
        self.label_sel = label_sel
        self.field_sel = field_sel
        self.index_value = index_value
        self.closed = False
        self.shard = None      # (index, count): scheduler-shard selection (api/sharding.py)
        self.bookmarks = False
        self._pending = None   # events coalesced until the end of this loop iteration
        self._loop = None
        self.pb = False        # protobuf watch stream (length-delimited WatchEvent frames)

    def event(self, etype, entry):
        return pb_event_bytes(etype, entry) if self.pb else event_bytes(etype, entry.raw)

    def matches(self, e: Entry) -> bool:
        if self.namespace and e.fields.get("metadata.namespace") != self.namespace:
            return False
        if self.label_sel is not None and not self.label_sel.matches(e.labels):
            return False
        if self.field_sel is not None and not self.field_sel.matches(e.fields):
            return False
        if self.shard is not None and not shard_matches(e.fields, e.labels, *self.shard):
            return False
        return True

    def send(self, data: bytes):
        if self.closed:
            return
        w = self.writer
        tr = w.transport
        if tr.is_closing():
            self.stop()
            return
        # slow-watcher protection (reference: cacher terminates watchers whose buffer is full)
        if tr.get_write_buffer_size() > 64 << 20:
            log.warning("terminating slow watcher on %s", self.cache.resource)
            self.stop()
            return
        # coalesce: all events dispatched in one event-loop iteration go out as ONE chunk /
        # one send() — under load this removes most per-event syscalls
        if self._pending is None:
            self._pending = [data]
            if self._loop is None:
                import asyncio
                self._loop = asyncio.get_event_loop()
            self._loop.call_soon(self._flush)
        else:
            self._pending.append(data)

    def _flush(self):
        p, self._pending = self._pending, None
        if p and not self.closed:
            self.writer.write(p[0] if len(p) == 1 else b"".join(p))

    def stop(self):
        if not self.closed:
            self.closed = True
            self.cache.remove_watcher(self)


def event_bytes(etype: str, raw: bytes) -> bytes:
    return b'{"type":"' + etype.encode() + b'","object":' + raw + b"}\n"


def pb_event_bytes(etype: str, entry: Entry) -> bytes:
    """One `application/vnd.kubernetes.protobuf;stream=watch` frame (watch.go:166-226)."""
    from ..api import protobuf as pb
    return pb.watch_frame(etype, entry.pb_envelope())


def error_event(status: dict, protobuf=False) -> bytes:
    if protobuf:
        from ..api import protobuf as pb
        return pb.watch_frame(ERROR, pb.status_envelope(status))
    return codec.dumpb({"type": ERROR, "object": status}) + b"\n"


class ResourceCache:
    def __init__(self, resource: str, window: int = 100_000):
        self.resource = resource
        self.fields_fn = FIELD_FUNCS.get(resource, generic_fields)
        self.by_key: dict[str, Entry] = {}
        self.events: deque = deque(maxlen=window)   # (rev, etype, entry, prev_entry)
        self.watchers: set[Watcher] = set()
        # watchers indexed by spec.nodeName (pods): kubelets watch only their node's pods
        self.indexed: dict[str, set[Watcher]] = {}
        self._unindexed: set[Watcher] = set()
        self.rev = 0

    # -- reads ------------------------------------------------------------
    def get(self, key):
        return self.by_key.get(key)

    def list(self, prefix: str, label_sel=None, field_sel=None):
        out = []
        for k, e in self.by_key.items():
            if not k.startswith(prefix):
                continue
            if label_sel is not None and not label_sel.matches(e.labels):
                continue
            if field_sel is not None and not field_sel.matches(e.fields):
                continue
            out.append(e)
        out.sort(key=lambda e: e.sort_key)
        return out

    # -- writes -----------------------------------------------------------
    def index_fields(self, obj):
        fields = self.fields_fn(obj)
        if ((obj.get("metadata") or {}).get("initializers") or {}).get("pending"):
            # alpha Initializers: uninitialized objects are hidden from list/watch unless the
            # client passes includeUninitialized=true (the server adds this field selector)
            fields = dict(fields, **{UNINITIALIZED: "true"})
        return fields

    def make_entry(self, obj, raw, rev):
        return Entry(obj, raw, rev, self.index_fields(obj))

    def apply(self, etype: str, key: str, entry: Entry, prev: Entry | None):
        """Record + dispatch one committed change (entry is the new state; for DELETED the
        final object state)."""
        self.rev = entry.rev
        if etype == DELETED:
            self.by_key.pop(key, None)
        else:
            self.by_key[key] = entry
        self.events.append((entry.rev, etype, entry, prev))
        if self.watchers:
            self._dispatch(etype, entry, prev)

    def _dispatch(self, etype, entry, prev):
        data = {}

        def enc(t, pbw=False):
            b = data.get((t, pbw))
            if b is None:
                b = data[(t, pbw)] = pb_event_bytes(t, entry) if pbw else event_bytes(t, entry.raw)
            return b

        if self.indexed:
            targets = set(self.indexed.get(entry.fields.get("spec.nodeName", ""), ()))
            if prev is not None:
                pv = prev.fields.get("spec.nodeName", "")
                if pv != entry.fields.get("spec.nodeName", ""):
                    targets |= self.indexed.get(pv, set())
            targets |= self._unindexed
        else:
            targets = self.watchers
        rev = entry.rev
        for w in list(targets):
            if w.closed or rev <= w.min_rev:
                continue
            cur = etype != DELETED and w.matches(entry)
            was = prev is not None and w.matches(prev)
            if etype == ADDED:
                if cur:
                    w.send(enc(ADDED, w.pb))
            elif etype == MODIFIED:
                if cur and was:
                    w.send(enc(MODIFIED, w.pb))
                elif cur:
                    w.send(enc(ADDED, w.pb))
                elif was:
                    w.send(enc(DELETED, w.pb))
            else:  # DELETED
                if w.matches(entry) or was:
                    w.send(enc(DELETED, w.pb))

    # -- watchers ---------------------------------------------------------
    def add_watcher(self, writer, namespace, label_selector, field_selector, from_rev: int | None, send_initial: bool,
                    shard=None, protobuf=False):
        ls = parse_labels(label_selector) if label_selector else None
        fs = parse_field_selector(field_selector) if field_selector else None
        idx = fs.requires("spec.nodeName") if (fs is not None and self.resource == "pods") else None
        w = Watcher(self, writer, namespace, ls, fs, idx)
        w.shard = shard
        w.pb = protobuf
        if from_rev is not None and not send_initial:
            w.min_rev = from_rev
        # initial state / replay (synchronous, so no event can interleave)
        if send_initial:
            for e in self.by_key.values():
                if w.matches(e):
                    w.send(w.event(ADDED, e))
        elif from_rev is not None:
            if self.events and from_rev < self.events[0][0] - 1 and len(self.events) == self.events.maxlen:
                raise GoneError(f"too old resource version: {from_rev} ({self.events[0][0] - 1})")
            for rev, etype, entry, prev in self.events:
                if rev <= from_rev:
                    continue
                cur = etype != DELETED and w.matches(entry)
                was = prev is not None and w.matches(prev)
                if etype == DELETED:
                    if w.matches(entry) or was:
                        w.send(w.event(DELETED, entry))
                elif cur:
                    w.send(w.event(MODIFIED if (was and etype == MODIFIED) else ADDED, entry))
                elif was:
                    w.send(w.event(DELETED, entry))
        self.watchers.add(w)
        if idx is not None:
            self.indexed.setdefault(idx, set()).add(w)
        elif self.resource == "pods":
            self._unindexed.add(w)
        return w

    def remove_watcher(self, w):
        self.watchers.discard(w)
        if w.index_value is not None:
            s = self.indexed.get(w.index_value)
            if s:
                s.discard(w)
                if not s:
                    del self.indexed[w.index_value]
        else:
            self._unindexed.discard(w)

    def decode_entry(self, raw, rev):
        return self.make_entry(codec.loads(raw), raw, rev)
