"""Typed REST client ("clientset") over `HTTPClient`.

Parity: client-go typed clients + `rest.Request` verbs (`staging/src/k8s.io/client-go/rest/request.go`),
client-side QPS/Burst token bucket (`util/flowcontrol`), `errors.IsNotFound/IsConflict/IsAlreadyExists`.
"""
from __future__ import annotations

import asyncio
import collections
import time
from urllib.parse import quote, urlencode

from ..api import codec, meta as m
from .http import HTTPClient


class APIStatusError(Exception):
    def __init__(self, code, status):
        self.code = code
        self.status = status if isinstance(status, dict) else {"message": str(status)}
        self.reason = self.status.get("reason", "")
        super().__init__(f"{code} {self.reason}: {self.status.get('message', '')}")


def is_not_found(e):
    return isinstance(e, APIStatusError) and e.code == 404


def is_conflict(e):
    return isinstance(e, APIStatusError) and e.code == 409 and e.reason == "Conflict"


def is_already_exists(e):
    return isinstance(e, APIStatusError) and e.code == 409 and e.reason == "AlreadyExists"


def is_gone(e):
    return isinstance(e, APIStatusError) and e.code == 410


class TokenBucket:
    def __init__(self, qps, burst):
        self.qps, self.burst = qps, burst
        self.tokens = burst
        self.t = time.monotonic()

    async def wait(self):
        while True:
            now = time.monotonic()
            self.tokens = min(self.burst, self.tokens + (now - self.t) * self.qps)
            self.t = now
            if self.tokens >= 1:
                self.tokens -= 1
                return
            await asyncio.sleep((1 - self.tokens) / self.qps)


def resource_path(resource, namespace=None, name=None, subresource="", watch=False):
    """`resource`: a registered name (plural, kind, short name) or a `ResourceInfo` (a resource
    found through discovery, e.g. a custom resource this process never registered)."""
    ri = resource if isinstance(resource, m.ResourceInfo) else m.lookup(resource)
    if ri is None:
        raise ValueError(f"unknown resource {resource!r}")
    base = "/api/v1" if not ri.group else f"/apis/{ri.group}/{ri.version}"
    p = base
    if watch:
        p += "/watch"
    if ri.namespaced and namespace:
        p += f"/namespaces/{quote(namespace)}"
    p += f"/{ri.plural}"
    if name:
        p += f"/{quote(name)}"
    if subresource:
        p += f"/{subresource}"
    return p


JSON, PROTOBUF = "application/json", "application/vnd.kubernetes.protobuf"


class Client:
    """`content_type` is the wire format (`--kube-api-content-type`, `rest.Config.ContentType`):
    with protobuf, objects of kinds the protobuf schema covers are sent protobuf-encoded and
    responses are asked for as protobuf (falling back to JSON per response, as the reference's
    negotiated serializer does — lists, CRs and Status bodies come back as JSON), and watches
    are protobuf streams (`application/vnd.kubernetes.protobuf;stream=watch`: length-delimited
    WatchEvent frames, decoded by the native codec)."""

    def __init__(self, url: str, token=None, qps: float | None = None, burst: int = 10, max_conns=16,
                 user_agent="kubernetes-amd", ssl_context=None, timeout=60.0, content_type=JSON):
        if content_type not in (JSON, PROTOBUF):
            raise ValueError(f"unsupported content type {content_type!r} (use {JSON} or {PROTOBUF})")
        self.url = url
        self.http = HTTPClient(url, token=token, ssl_context=ssl_context, max_conns=max_conns, timeout=timeout)
        self.limiter = TokenBucket(qps, burst) if qps else None
        self.user_agent = user_agent
        self.content_type = content_type
        self._accept = {"Accept": f"{PROTOBUF}, {JSON}"} if content_type == PROTOBUF else None

    @staticmethod
    def _decode(resp):
        if resp[:4] == b"k8s\x00":
            from ..api import protobuf as pb
            return pb.decode_object(resp)
        return codec.loads(resp)

    async def close(self):
        await self.http.close()

    async def _do(self, method, path, body=None, content_type="application/json", ok=(200, 201), decode=True):
        """`decode=False`: the caller ignores the response object (an event write, a final
        delete, a binding): skip parsing it; errors are still decoded."""
        if self.limiter:
            await self.limiter.wait()
        if body is None or isinstance(body, (bytes, bytearray)):
            data = body
        elif self._accept is not None and content_type == JSON and body.get("kind"):
            from ..api import protobuf as pb
            if pb.supported(body["kind"], body.get("apiVersion") or "v1"):
                data, content_type = pb.encode_object(body), PROTOBUF
            else:
                data = codec.dumpb(body)
        else:
            data = codec.dumpb(body)
        st, resp = await self.http.request(method, path, data, content_type, self._accept)
        if st not in ok:
            try:
                status = self._decode(resp)
            except Exception:
                status = {"message": resp.decode(errors="replace")}
            raise APIStatusError(st, status)
        return self._decode(resp) if resp and decode else None

    async def raw(self, method, path, body=None, content_type="application/json"):
        return await self.http.request(method, path, body, content_type)

    # -- verbs -----------------------------------------------------------
    async def get(self, resource, name, namespace=None, subresource=""):
        return await self._do("GET", resource_path(resource, namespace, name, subresource))

    async def list(self, resource, namespace=None, label_selector=None, field_selector=None, limit=0,
                   cont=None, resource_version=None, extra=None):
        q = dict(extra or {})
        if label_selector:
            q["labelSelector"] = label_selector
        if field_selector:
            q["fieldSelector"] = field_selector
        if limit:
            q["limit"] = str(limit)
        if cont:
            q["continue"] = cont
        if resource_version is not None:
            q["resourceVersion"] = resource_version
        path = resource_path(resource, namespace)
        if q:
            path += "?" + urlencode(q)
        return await self._do("GET", path)

    async def list_all(self, resource, namespace=None, label_selector=None, field_selector=None, chunk=500,
                       extra=None):
        out, cont, rv = [], None, None
        while True:
            lst = await self.list(resource, namespace, label_selector, field_selector, limit=chunk, cont=cont,
                                  extra=extra)
            out.extend(lst.get("items") or [])
            rv = lst["metadata"].get("resourceVersion")
            cont = lst["metadata"].get("continue")
            if not cont:
                return out, rv

    async def create(self, resource, obj, namespace=None, decode=True):
        ns = namespace or (obj.get("metadata") or {}).get("namespace")
        return await self._do("POST", resource_path(resource, ns), obj, decode=decode)

    async def update(self, resource, obj, namespace=None, subresource=""):
        md = obj.get("metadata") or {}
        ns = namespace or md.get("namespace")
        return await self._do("PUT", resource_path(resource, ns, md["name"], subresource), obj)

    async def update_status(self, resource, obj, namespace=None):
        return await self.update(resource, obj, namespace, "status")

    async def patch(self, resource, name, patch, namespace=None, patch_type="merge", subresource="", decode=True):
        ct = {"merge": "application/merge-patch+json", "strategic": "application/strategic-merge-patch+json",
              "json": "application/json-patch+json"}[patch_type]
        return await self._do("PATCH", resource_path(resource, namespace, name, subresource), patch, ct, decode=decode)

    async def delete(self, resource, name, namespace=None, grace_period=None, propagation=None, uid=None,
                     decode=True):
        opts = {"kind": "DeleteOptions", "apiVersion": "v1"}
        if grace_period is not None:
            opts["gracePeriodSeconds"] = grace_period
        if propagation:
            opts["propagationPolicy"] = propagation
        if uid:
            opts["preconditions"] = {"uid": uid}
        return await self._do("DELETE", resource_path(resource, namespace, name), opts, decode=decode)

    async def delete_collection(self, resource, namespace=None, label_selector=None):
        path = resource_path(resource, namespace)
        if label_selector:
            path += "?" + urlencode({"labelSelector": label_selector})
        return await self._do("DELETE", path)

    async def bind(self, namespace, name, node, extended_resource_binding=None, annotations=None, uid=None,
                   decode=True):
        target = {"kind": "Node", "apiVersion": "v1", "name": node}
        if extended_resource_binding:
            target["extendedResourceBinding"] = extended_resource_binding
        body = {"kind": "Binding", "apiVersion": "v1", "metadata": {"name": name, "namespace": namespace},
                "target": target}
        if annotations:
            body["metadata"]["annotations"] = annotations
        if uid:
            body["metadata"]["uid"] = uid
        return await self._do("POST", resource_path("pods", namespace, name, "binding"), body, decode=decode)

    async def evict(self, namespace, name, grace_period=None):
        body = {"kind": "Eviction", "apiVersion": "policy/v1beta1", "metadata": {"name": name, "namespace": namespace}}
        if grace_period is not None:
            body["deleteOptions"] = {"gracePeriodSeconds": grace_period}
        return await self._do("POST", resource_path("pods", namespace, name, "eviction"), body)

    async def watch(self, resource, namespace=None, resource_version=None, label_selector=None,
                    field_selector=None, timeout_seconds=None, extra=None):
        """Async iterator of (event_type, object). Closes when the server ends the stream.
        `extra`: additional query parameters (e.g. {"kamdShard": "i/n"})."""
        q = dict(extra or {})
        q["watch"] = "true"
        if resource_version is not None:
            q["resourceVersion"] = str(resource_version)
        if label_selector:
            q["labelSelector"] = label_selector
        if field_selector:
            q["fieldSelector"] = field_selector
        if timeout_seconds:
            q["timeoutSeconds"] = str(int(timeout_seconds))
        path = resource_path(resource, namespace) + "?" + urlencode(q)
        headers, frames = None, None
        if self._accept is not None:
            # protobuf watch streams (the reference client negotiates the same): length-delimited
            # WatchEvent frames decoded natively; the server answers JSON for kinds protobuf
            # cannot carry (custom resources)
            from ..api import protobuf as pb
            headers = {"Accept": f"{PROTOBUF}, {JSON}"}
            frames = pb.decode_watch_frames
        try:
            _, lines, closer, ctype = await self.http.stream("GET", path, headers, frames)
        except Exception as e:
            from .http import HTTPError
            if isinstance(e, HTTPError):
                try:
                    st = codec.loads(e.body)
                except Exception:
                    st = {"message": e.body.decode(errors="replace")}
                raise APIStatusError(e.status, st)
            raise
        return _WatchStream(lines, closer, frames is not None and "protobuf" in ctype)


def _event(line):
    ev = codec.loads(line)
    if ev.get("type") == "ERROR":
        obj = ev.get("object") or {}
        raise APIStatusError(obj.get("code", 500), obj)
    return ev["type"], ev["object"]


def _pb_event(ev):
    """An already-decoded protobuf watch event (type, object)."""
    if ev[0] == "ERROR":
        obj = ev[1] or {}
        raise APIStatusError(obj.get("code", 500), obj)
    return ev

class _WatchStream:
    """Watch events, one at a time (`async for typ, obj in stream`) or per received batch
    (`async for evs in stream.batches()`, what informers use: one await per network read)."""

    def __init__(self, batches, closer, protobuf=False):
        self._batches = batches
        self._closer = closer
        self._pending = collections.deque()
        self._ev = _pb_event if protobuf else _event
        self.protobuf = protobuf

    def __aiter__(self):
        return self

    async def __anext__(self):
        while not self._pending:
            self._pending.extend(await self._batches.__anext__())
        return self._ev(self._pending.popleft())

    async def batches(self):
        ev = self._ev
        if self._pending:
            lines, self._pending = list(self._pending), collections.deque()
            yield [ev(ln) for ln in lines]
        async for lines in self._batches:
            out = []
            for ln in lines:
                try:
                    out.append(ev(ln))
                except APIStatusError:
                    if out:
                        yield out
                    raise
            yield out

    def close(self):
        self._closer()
