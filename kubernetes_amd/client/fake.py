"""In-memory fake client for controller unit tests.

Parity: `staging/src/k8s.io/client-go/kubernetes/fake` + `client-go/testing/fixture.go`
(`ObjectTracker`: objects by resource/namespace/name with resourceVersions and watch fan-out)
and `client-go/testing/fake.go` (`Fake.Actions()` records every call; `PrependReactor(verb,
resource, fn)` lets a test intercept calls — return `(True, result)` to answer, raise to fail,
`(False, None)` to fall through to the tracker).

`FakeClient` has the async surface of `client.rest.Client` (get / list / create / update /
update_status / patch / delete / bind / evict / watch), so informers and controllers run on it
unchanged.
"""
from __future__ import annotations

import asyncio
import copy
import itertools
import uuid

from ..api import meta as m
from ..api.labels import parse as parse_selector
from ..api.meta import now_rfc3339
from ..utils.patch import apply_patch
from .rest import APIStatusError

_PATCH_TYPES = {"merge": "application/merge-patch+json", "strategic": "application/strategic-merge-patch+json",
                "json": "application/json-patch+json"}


def _plural(resource):
    return resource.plural if isinstance(resource, m.ResourceInfo) else resource


def _status(code, reason, msg):
    return APIStatusError(code, {"kind": "Status", "apiVersion": "v1", "status": "Failure", "code": code,
                                 "reason": reason, "message": msg})


class Action:
    __slots__ = ("verb", "resource", "namespace", "name", "subresource", "obj")

    def __init__(self, verb, resource, namespace=None, name=None, subresource="", obj=None):
        self.verb, self.resource, self.namespace, self.name, self.subresource, self.obj = \
            verb, resource, namespace, name, subresource, obj

    def __repr__(self):
        return f"Action({self.verb} {self.resource}{'/' + self.subresource if self.subresource else ''} " \
               f"{self.namespace or ''}/{self.name or ''})"


class _FakeWatch:
    def __init__(self, q, on_close):
        self.q, self._on_close = q, on_close

    def __aiter__(self):
        return self

    async def __anext__(self):
        ev = await self.q.get()
        if ev is None:
            raise StopAsyncIteration
        return ev

    async def batches(self):
        """Same contract as the real stream: lists of events (everything queued so far)."""
        while True:
            ev = await self.q.get()
            if ev is None:
                return
            out = [ev]
            while not self.q.empty():
                nxt = self.q.get_nowait()
                if nxt is None:
                    yield out
                    return
                out.append(nxt)
            yield out

    def close(self):
        self._on_close(self.q)
        self.q.put_nowait(None)


class FakeClient:
    def __init__(self, *objects):
        self.objects: dict[str, dict[tuple, dict]] = {}
        self.rv = itertools.count(1)
        self.actions: list[Action] = []
        self.reactors: list[tuple] = []
        self.watchers: dict[str, list] = {}
        for o in objects:
            ri = m.BY_KIND[o["kind"]]
            self._store(ri.plural, copy.deepcopy(o))

    # -- test hooks ----------------------------------------------------------------------
    def prepend_reactor(self, verb, resource, fn):
        self.reactors.insert(0, (verb, resource, fn))

    def clear_actions(self):
        self.actions.clear()

    def _react(self, action):
        if isinstance(action.resource, m.ResourceInfo):
            action.resource = action.resource.plural
        self.actions.append(action)
        for verb, res, fn in self.reactors:
            if verb in ("*", action.verb) and res in ("*", action.resource):
                handled, result = fn(action)
                if handled:
                    return True, result
        return False, None

    # -- tracker -------------------------------------------------------------------------
    def _key(self, plural, ns, name):
        plural = _plural(plural)
        ri = m.BY_PLURAL.get(plural)
        return ((ns or "default") if ri is None or ri.namespaced else None, name)

    def _store(self, plural, obj, event="ADDED"):
        md = obj.setdefault("metadata", {})
        md["resourceVersion"] = str(next(self.rv))
        md.setdefault("uid", str(uuid.uuid4()))
        md.setdefault("creationTimestamp", now_rfc3339())
        ri = m.BY_PLURAL.get(plural)
        if ri is not None:
            obj.setdefault("kind", ri.kind)
            obj.setdefault("apiVersion", ri.group_version)
            if ri.namespaced:
                md.setdefault("namespace", "default")
        self.objects.setdefault(plural, {})[self._key(plural, md.get("namespace"), md["name"])] = obj
        self._notify(plural, event, obj)
        return copy.deepcopy(obj)

    def _notify(self, plural, typ, obj):
        for ns, q in list(self.watchers.get(plural, ())):
            if ns is None or obj["metadata"].get("namespace") == ns:
                q.put_nowait((typ, copy.deepcopy(obj)))

    def _get(self, plural, name, ns):
        o = self.objects.get(plural, {}).get(self._key(plural, ns, name))
        if o is None:
            raise _status(404, "NotFound", f'{plural} "{name}" not found')
        return o

    # -- client surface ------------------------------------------------------------------
    async def close(self):
        for plural, lst in self.watchers.items():
            for _, q in lst:
                q.put_nowait(None)

    async def get(self, resource, name, namespace=None, subresource=""):
        resource = _plural(resource)
        h, r = self._react(Action("get", resource, namespace, name, subresource))
        if h:
            return r
        return copy.deepcopy(self._get(resource, name, namespace))

    async def list(self, resource, namespace=None, label_selector=None, field_selector=None, limit=0, continue_=None,
                   **_kw):
        resource = _plural(resource)
        h, r = self._react(Action("list", resource, namespace))
        if h:
            return r
        sel = parse_selector(label_selector) if label_selector else None
        items = []
        for (ns, _), o in sorted(self.objects.get(resource, {}).items(), key=lambda kv: (kv[0][0] or "", kv[0][1])):
            if namespace is not None and ns != namespace:
                continue
            if sel is not None and not sel.matches(o["metadata"].get("labels") or {}):
                continue
            if field_selector:
                ok = True
                for term in field_selector.split(","):
                    neg = "!=" in term
                    k, v = term.split("!=" if neg else "=", 1)
                    cur = o
                    for part in k.split("."):
                        cur = (cur or {}).get(part) if isinstance(cur, dict) else None
                    if (str(cur if cur is not None else "") == v) == neg:
                        ok = False
                if not ok:
                    continue
            items.append(copy.deepcopy(o))
        ri = m.BY_PLURAL.get(resource)
        return {"kind": (ri.kind if ri else "") + "List", "apiVersion": ri.group_version if ri else "v1",
                "metadata": {"resourceVersion": str(next(self.rv))}, "items": items}

    async def list_all(self, resource, namespace=None, label_selector=None, field_selector=None, chunk=500, **_kw):
        resource = _plural(resource)
        lst = await self.list(resource, namespace, label_selector, field_selector)
        return lst["items"], lst["metadata"]["resourceVersion"]

    async def create(self, resource, obj, namespace=None, decode=True):
        resource = _plural(resource)
        obj = copy.deepcopy(obj)
        md = obj.setdefault("metadata", {})
        if namespace and m.BY_PLURAL.get(resource, m.BY_PLURAL["pods"]).namespaced:
            md["namespace"] = namespace
        if not md.get("name") and md.get("generateName"):
            md["name"] = md["generateName"] + uuid.uuid4().hex[:5]
        h, r = self._react(Action("create", resource, md.get("namespace"), md.get("name"), "", obj))
        if h:
            return r
        if self._key(resource, md.get("namespace"), md["name"]) in self.objects.get(resource, {}):
            raise _status(409, "AlreadyExists", f'{resource} "{md["name"]}" already exists')
        return self._store(resource, obj)

    async def update(self, resource, obj, namespace=None, subresource=""):
        resource = _plural(resource)
        obj = copy.deepcopy(obj)
        md = obj["metadata"]
        ns = namespace or md.get("namespace")
        h, r = self._react(Action("update", resource, ns, md["name"], subresource, obj))
        if h:
            return r
        cur = self._get(resource, md["name"], ns)
        if md.get("resourceVersion") and md["resourceVersion"] != cur["metadata"]["resourceVersion"]:
            raise _status(409, "Conflict", "the object has been modified; please apply your changes to the latest version")
        md["uid"] = cur["metadata"]["uid"]
        md["creationTimestamp"] = cur["metadata"].get("creationTimestamp")
        if subresource == "status":
            new = copy.deepcopy(cur)
            new["status"] = obj.get("status")
            obj = new
        return self._store(resource, obj, "MODIFIED")

    async def update_status(self, resource, obj, namespace=None):
        return await self.update(resource, obj, namespace, "status")

    async def patch(self, resource, name, patch, namespace=None, patch_type="merge", subresource="", decode=True):
        resource = _plural(resource)
        h, r = self._react(Action("patch", resource, namespace, name, subresource, patch))
        if h:
            return r
        cur = copy.deepcopy(self._get(resource, name, namespace))
        new = apply_patch(_PATCH_TYPES.get(patch_type, patch_type), cur, patch)
        return self._store(resource, new, "MODIFIED")

    async def delete(self, resource, name, namespace=None, grace_period=None, propagation=None, uid=None,
                     decode=True):
        resource = _plural(resource)
        h, r = self._react(Action("delete", resource, namespace, name))
        if h:
            return r
        o = self._get(resource, name, namespace)
        if uid and o["metadata"]["uid"] != uid:
            raise _status(409, "Conflict", "Precondition failed: UID in precondition does not match")
        del self.objects[resource][self._key(resource, namespace, name)]
        self._notify(resource, "DELETED", o)
        return {"kind": "Status", "status": "Success"}

    async def delete_collection(self, resource, namespace=None, label_selector=None):
        resource = _plural(resource)
        for o in (await self.list(resource, namespace, label_selector))["items"]:
            await self.delete(resource, o["metadata"]["name"], o["metadata"].get("namespace"))

    async def bind(self, namespace, name, node, extended_resource_binding=None, annotations=None, uid=None,
                   decode=True):
        h, r = self._react(Action("create", "pods", namespace, name, "binding",
                                  {"target": {"name": node}, "extendedResources": extended_resource_binding}))
        if h:
            return r
        pod = copy.deepcopy(self._get("pods", name, namespace))
        if pod["spec"].get("nodeName"):
            raise _status(409, "Conflict", f"pod {name} is already assigned to node {pod['spec']['nodeName']}")
        pod["spec"]["nodeName"] = node
        for per in pod["spec"].get("extendedResources") or ():
            got = (extended_resource_binding or {}).get(per.get("name"))
            if got:
                per["assigned"] = list(got["resources"])
        self._store("pods", pod, "MODIFIED")
        return {"kind": "Status", "status": "Success"}

    async def evict(self, namespace, name, grace_period=None):
        h, r = self._react(Action("create", "pods", namespace, name, "eviction"))
        if h:
            return r
        return await self.delete("pods", name, namespace)

    async def watch(self, resource, namespace=None, resource_version=None, label_selector=None, field_selector=None,
                    timeout_seconds=None, **_kw):
        resource = _plural(resource)
        self._react(Action("watch", resource, namespace))
        q: asyncio.Queue = asyncio.Queue()
        ent = (namespace, q)
        self.watchers.setdefault(resource, []).append(ent)

        def remove(qq):
            lst = self.watchers.get(resource, [])
            self.watchers[resource] = [e for e in lst if e[1] is not qq]
        return _FakeWatch(q, remove)
