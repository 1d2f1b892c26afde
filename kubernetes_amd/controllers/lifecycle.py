"""Lifecycle controllers: namespace deletion, garbage collection, pod GC, node lifecycle.

Parity:
  * NamespaceController — `pkg/controller/namespace/deletion/namespaced_resources_deleter.go`:
    a Terminating namespace has all its namespaced content deleted, then its `kubernetes`
    finalizer is removed through `/finalize` and the namespace disappears.
  * GarbageCollector — `pkg/controller/garbagecollector`: dependents whose owner (by UID) is
    gone are deleted (background); `orphan` finalizer strips ownerReferences from dependents;
    `foregroundDeletion` deletes dependents first, then releases the owner.
  * PodGC — `pkg/controller/podgc/gc_controller.go`: terminated pods above
    `terminated_pod_gc_threshold` (oldest first) and pods bound to nodes that no longer exist.
  (Node lifecycle — health, zones, rate-limited evictions, taint manager — is in
  `nodelifecycle.py`.)
"""
from __future__ import annotations

import asyncio
import time

from ..api import core, meta as m
from ..api.meta import now_rfc3339
from ..client.rest import APIStatusError, is_conflict, is_not_found
from .base import Controller, split_key

class NamespaceController(Controller):
    name = "namespace"
    primary = "namespaces"
    workers = 2

    def setup(self):
        self.ns_inf = self.factory.get("namespaces")
        self.ns_inf.add_handler(self._maybe, lambda o, n: self._maybe(n), None)

    def _maybe(self, ns):
        if ns["metadata"].get("deletionTimestamp"):
            self.enqueue(ns["metadata"]["name"])

    async def sync(self, key):
        ns = self.ns_inf.get(key)
        if ns is None or not ns["metadata"].get("deletionTimestamp"):
            return
        name = ns["metadata"]["name"]
        remaining = 0
        for ri in m.RESOURCES:
            if not ri.namespaced:
                continue
            try:
                lst = await self.client.list(ri.plural, name)
            except APIStatusError:
                continue
            for o in lst.get("items") or ():
                remaining += 1
                if o["metadata"].get("deletionTimestamp") and ri.plural != "pods":
                    continue
                try:
                    await self.client.delete(ri.plural, o["metadata"]["name"], name,
                                             grace_period=0 if ri.plural != "pods" else None)
                except APIStatusError as e:
                    if not is_not_found(e):
                        raise
        if remaining:
            self.queue.add_after(key, 0.2)   # wait for graceful pod deletion, then finalize
            return
        fins = [f for f in (ns.get("spec") or {}).get("finalizers") or [] if f != "kubernetes"]
        st, body = await self.client.raw("PUT", f"/api/v1/namespaces/{name}/finalize",
                                         _dump({"metadata": {"name": name}, "spec": {"finalizers": fins}}))
        if st not in (200, 404):
            raise RuntimeError(f"finalize {name}: {st} {body[:200]!r}")


def _dump(o):
    from ..api import codec
    return codec.dumpb(o)


class GarbageCollector(Controller):
    """Owner-reference graph over the informer caches of every served resource."""
    name = "garbagecollector"
    workers = 4
    RESOURCES = ("pods", "replicasets", "deployments", "jobs", "cronjobs", "daemonsets", "statefulsets",
                 "replicationcontrollers", "controllerrevisions", "configmaps", "secrets", "services",
                 "endpoints", "poddisruptionbudgets")

    def setup(self):
        self.infs = {r: self.factory.get(r) for r in self.RESOURCES}
        self.uids: dict[str, tuple] = {}          # uid -> (resource, key)
        self.children: dict[str, set] = {}        # owner uid -> {(resource, key)}
        for r, inf in self.infs.items():
            inf.add_handler(lambda o, r=r: self._add(r, o), lambda old, new, r=r: self._update(r, old, new),
                            lambda o, r=r: self._delete(r, o))

    def _refs(self, o):
        return [ref["uid"] for ref in (o["metadata"].get("ownerReferences") or ()) if ref.get("uid")]

    def _add(self, r, o):
        key = m.ns_name(o)
        uid = o["metadata"].get("uid")
        self.uids[uid] = (r, key)
        for ou in self._refs(o):
            self.children.setdefault(ou, set()).add((r, key))
            if ou not in self.uids:
                self.enqueue(f"dep|{r}|{key}")
        fins = o["metadata"].get("finalizers") or ()
        if o["metadata"].get("deletionTimestamp") and ("orphan" in fins or "foregroundDeletion" in fins):
            self.enqueue(f"own|{r}|{key}")

    def _update(self, r, old, new):
        for ou in self._refs(old):
            s = self.children.get(ou)
            if s:
                s.discard((r, m.ns_name(old)))
        self._add(r, new)

    def _delete(self, r, o):
        uid = o["metadata"].get("uid")
        self.uids.pop(uid, None)
        for ou in self._refs(o):
            s = self.children.get(ou)
            if s:
                s.discard((r, m.ns_name(o)))
        for child in list(self.children.get(uid, ())):
            self.enqueue(f"dep|{child[0]}|{child[1]}")
        owner_fg = [ou for ou in self._refs(o) if ou in self.uids]
        for ou in owner_fg:
            r2, k2 = self.uids[ou]
            self.enqueue(f"own|{r2}|{k2}")

    async def sync(self, key):
        kind, r, okey = key.split("|", 2)
        obj = self.infs[r].get(okey)
        if obj is None:
            return
        ns, name = split_key(okey)
        if kind == "dep":
            refs = obj["metadata"].get("ownerReferences") or []
            if not refs:
                return
            alive = [ref for ref in refs if ref.get("uid") in self.uids]
            if alive:
                # owner still exists; if it is being deleted in the foreground, delete the dependent
                for ref in alive:
                    r2, k2 = self.uids[ref["uid"]]
                    owner = self.infs[r2].get(k2)
                    if owner and owner["metadata"].get("deletionTimestamp") and "foregroundDeletion" in (owner["metadata"].get("finalizers") or ()):
                        await self._del(r, name, ns)
                return
            await self._del(r, name, ns)
            return
        # owner with orphan / foreground finalizer
        fins = list(obj["metadata"].get("finalizers") or [])
        uid = obj["metadata"]["uid"]
        kids = [c for c in self.children.get(uid, ()) if self.infs[c[0]].get(c[1]) is not None]
        if "orphan" in fins:
            for cr, ck in kids:
                child = self.infs[cr].get(ck)
                refs = [x for x in child["metadata"].get("ownerReferences") or () if x.get("uid") != uid]
                cns, cname = split_key(ck)
                try:
                    await self.client.patch(cr, cname, {"metadata": {"ownerReferences": refs or None}}, cns)
                except APIStatusError as e:
                    if not is_not_found(e):
                        raise
            fins.remove("orphan")
        elif "foregroundDeletion" in fins:
            if kids:
                for cr, ck in kids:
                    cns, cname = split_key(ck)
                    await self._del(cr, cname, cns)
                self.queue.add_after(key, 0.2)
                return
            fins.remove("foregroundDeletion")
        else:
            return
        try:
            await self.client.patch(r, name, {"metadata": {"finalizers": fins or None}}, ns)
        except APIStatusError as e:
            if not (is_not_found(e) or is_conflict(e)):
                raise

    async def _del(self, r, name, ns):
        try:
            await self.client.delete(r, name, ns, propagation="Background")
        except APIStatusError as e:
            if not is_not_found(e):
                raise


class PodGCController(Controller):
    name = "podgc"
    workers = 1

    def __init__(self, client, factory, recorder=None, terminated_pod_gc_threshold=12500, period=20.0):
        super().__init__(client, factory, recorder)
        self.threshold = terminated_pod_gc_threshold
        self.period = period
        self._tick = None

    def setup(self):
        self.pod_inf = self.factory.get("pods")
        self.node_inf = self.factory.get("nodes")

    def start(self):
        super().start()
        self._tick = asyncio.ensure_future(self._ticker())

    def stop(self):
        super().stop()
        if self._tick:
            self._tick.cancel()

    async def _ticker(self):
        while True:
            await asyncio.sleep(self.period)
            self.enqueue("gc")

    async def sync(self, key):
        pods = self.pod_inf.list()
        term = [p for p in pods if core.pod_is_terminal(p)]
        if len(term) > self.threshold:
            term.sort(key=lambda p: p["metadata"].get("creationTimestamp", ""))
            for p in term[:len(term) - self.threshold]:
                await self._force(p)
        nodes = {n["metadata"]["name"] for n in self.node_inf.list()}
        for p in pods:
            nn = (p.get("spec") or {}).get("nodeName")
            if nn and nn not in nodes and self.node_inf.has_synced():
                await self._force(p)

    async def _force(self, p):
        try:
            await self.client.delete("pods", p["metadata"]["name"], p["metadata"]["namespace"], grace_period=0)
        except APIStatusError as e:
            if not is_not_found(e):
                raise


from .nodelifecycle import NodeLifecycleController  # noqa: E402,F401  (re-export)
