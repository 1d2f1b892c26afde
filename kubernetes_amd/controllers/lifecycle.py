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
  * NodeLifecycle — `pkg/controller/node/node_controller.go:420-916`: a node whose kubelet has
    not posted status for `grace` seconds gets Ready=Unknown plus the `unreachable` NoExecute
    taint; after `pod_eviction_timeout` its pods are evicted (deleted) unless they tolerate the
    taint longer (`tolerationSeconds`). GPU pods evicted here free their device IDs.
"""
from __future__ import annotations

import asyncio
import time

from ..api import core, meta as m
from ..api.meta import now_rfc3339
from ..client.rest import APIStatusError, is_conflict, is_not_found
from .base import Controller, split_key

UNREACHABLE_TAINT = "node.alpha.kubernetes.io/unreachable"
NOT_READY_TAINT = "node.alpha.kubernetes.io/notReady"


class NamespaceController(Controller):
    name = "namespace"
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


class NodeLifecycleController(Controller):
    name = "nodelifecycle"
    workers = 2

    def __init__(self, client, factory, recorder=None, monitor_period=5.0, grace=40.0, pod_eviction_timeout=300.0):
        super().__init__(client, factory, recorder)
        self.monitor_period = monitor_period
        self.grace = grace
        self.eviction_timeout = pod_eviction_timeout
        self._tick = None
        self.observed: dict[str, tuple] = {}   # node -> (heartbeat string, local time it changed)

    def setup(self):
        self.node_inf = self.factory.get("nodes")
        self.pod_inf = self.factory.get("pods")
        if "nodeName" not in self.pod_inf.store.indexers:
            self.pod_inf.store.add_indexer("nodeName", lambda p: [(p.get("spec") or {}).get("nodeName", "")])

    def start(self):
        super().start()
        self._tick = asyncio.ensure_future(self._ticker())

    def stop(self):
        super().stop()
        if self._tick:
            self._tick.cancel()

    async def _ticker(self):
        while True:
            await asyncio.sleep(self.monitor_period)
            for n in self.node_inf.list():
                self.enqueue(n["metadata"]["name"])

    async def sync(self, key, now=None):
        node = self.node_inf.get(key)
        if node is None:
            self.observed.pop(key, None)
            return
        now = now or time.monotonic()
        ready = core.get_condition(node.get("status"), "Ready")
        hb = (ready or {}).get("lastHeartbeatTime", "")
        prev = self.observed.get(key)
        if prev is None or prev[0] != hb:
            self.observed[key] = (hb, now)
            prev = self.observed[key]
        stale = now - prev[1] > self.grace
        taints = list((node.get("spec") or {}).get("taints") or [])
        has_taint = any(t.get("key") == UNREACHABLE_TAINT for t in taints)
        if stale:
            if ready is None or ready.get("status") != "Unknown":
                conds = []
                for c in (node.get("status") or {}).get("conditions") or ():
                    c = dict(c)
                    c["status"] = "Unknown"
                    c["reason"] = "NodeStatusUnknown"
                    c["message"] = "Kubelet stopped posting node status."
                    c["lastTransitionTime"] = now_rfc3339()
                    conds.append(c)
                await self._patch_status(key, conds)
                self.recorder.event(node, "Normal", "NodeNotReady", f"Node {key} status is now: NodeNotReady")
            if not has_taint:
                taints.append({"key": UNREACHABLE_TAINT, "effect": "NoExecute", "timeAdded": now_rfc3339()})
                await self.client.patch("nodes", key, {"spec": {"taints": taints}})
            # evict pods that do not tolerate the taint past their tolerationSeconds
            taint = {"key": UNREACHABLE_TAINT, "effect": "NoExecute"}
            for p in self.pod_inf.store.by_index("nodeName", key):
                if core.pod_is_terminal(p) or p["metadata"].get("deletionTimestamp"):
                    continue
                tol = [t for t in (p.get("spec") or {}).get("tolerations") or () if core.tolerates([t], taint)]
                limit = self.eviction_timeout if not tol else min(
                    (t.get("tolerationSeconds") if t.get("tolerationSeconds") is not None else float("inf")) for t in tol)
                if now - prev[1] - self.grace >= limit:
                    try:
                        await self.client.delete("pods", p["metadata"]["name"], p["metadata"]["namespace"])
                        self.recorder.event(p, "Normal", "TaintManagerEviction", f"Marking for deletion Pod {m.ns_name(p)}")
                    except APIStatusError as e:
                        if not is_not_found(e):
                            raise
        elif has_taint and ready is not None and ready.get("status") == "True":
            taints = [t for t in taints if t.get("key") != UNREACHABLE_TAINT]
            await self.client.patch("nodes", key, {"spec": {"taints": taints or None}})

    async def _patch_status(self, name, conds):
        try:
            await self.client.patch("nodes", name, {"status": {"conditions": conds}}, None, "merge", "status")
        except APIStatusError as e:
            if not is_not_found(e):
                raise
