"""Lifecycle controllers: namespace deletion, garbage collection, pod GC, node lifecycle.

Parity:
  * NamespaceController — `pkg/controller/namespace/deletion/namespaced_resources_deleter.go`:
    a Terminating namespace has all its namespaced content deleted, then its `kubernetes`
    finalizer is removed through `/finalize` and the namespace disappears.
  * GarbageCollector — `pkg/controller/garbagecollector`: in `garbagecollector.py`.
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

    async def namespaced_resources(self):
        """Every namespaced resource that supports list + delete, from discovery (custom
        resources included — `namespaced_resources_deleter.go` uses the discovery client too);
        the compiled-in set when discovery is unavailable."""
        if hasattr(self.client, "raw"):
            from .garbagecollector import discover
            try:
                lists = await discover(self.client)
            except (APIStatusError, OSError, ConnectionError):
                lists = None
            if lists:
                out, seen = [], set()
                for rl in lists:
                    gv = rl.get("groupVersion") or ""
                    group, _, version = gv.rpartition("/")
                    for r in rl.get("resources") or ():
                        name = r.get("name") or ""
                        if "/" in name or not r.get("namespaced") or (group, name) in seen:
                            continue
                        seen.add((group, name))
                        if not {"list", "delete"}.issubset(r.get("verbs") or ()):
                            continue
                        canon = m.BY_PLURAL.get(name) if (group, version, name) in m.ALIASES else None
                        if canon is not None and canon.group != group:
                            continue
                        if group == "" and name == "events":
                            continue            # events go last, with the namespace
                        out.append(m.ResourceInfo(group, version, r.get("kind") or "", name, True))
                return out
        return [ri for ri in m.RESOURCES if ri.namespaced and ri.plural not in m.VIRTUAL]

    async def sync(self, key):
        ns = self.ns_inf.get(key)
        if ns is None or not ns["metadata"].get("deletionTimestamp"):
            return
        name = ns["metadata"]["name"]
        remaining = 0
        for ri in await self.namespaced_resources():
            handle = ri.plural if (m.BY_PLURAL.get(ri.plural) or ri).group == ri.group else ri
            try:
                lst = await self.client.list(handle, name)
            except APIStatusError:
                continue
            for o in lst.get("items") or ():
                remaining += 1
                if o["metadata"].get("deletionTimestamp") and ri.plural != "pods":
                    continue
                try:
                    await self.client.delete(handle, o["metadata"]["name"], name,
                                             grace_period=0 if ri.plural != "pods" else None)
                except APIStatusError as e:
                    if not is_not_found(e):
                        raise
        if remaining:
            self.queue.add_after(key, 0.2)   # wait for graceful pod deletion, then finalize
            return
        try:
            await self.client.delete_collection("events", name)
        except APIStatusError:
            pass
        fins = [f for f in (ns.get("spec") or {}).get("finalizers") or [] if f != "kubernetes"]
        st, body = await self.client.raw("PUT", f"/api/v1/namespaces/{name}/finalize",
                                         _dump({"metadata": {"name": name}, "spec": {"finalizers": fins}}))
        if st not in (200, 404):
            raise RuntimeError(f"finalize {name}: {st} {body[:200]!r}")


def _dump(o):
    from ..api import codec
    return codec.dumpb(o)


class PodGCController(Controller):
    """`pkg/controller/podgc/gc_controller.go`, every 20 s: `gcTerminated` (the oldest
    terminated pods beyond `--terminated-pod-gc-threshold`; <= 0 disables it), `gcOrphaned`
    (pods bound to a node that no longer exists, checked against a live node list) and
    `gcUnscheduledTerminating` (terminating pods that were never scheduled: no kubelet will
    finish their deletion) — all force-deleted (grace period 0)."""
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
        if self.threshold > 0:
            term = [p for p in pods if core.pod_is_terminal(p)]
            if len(term) > self.threshold:
                term.sort(key=lambda p: p["metadata"].get("creationTimestamp", ""))
                await asyncio.gather(*(self._force(p) for p in term[:len(term) - self.threshold]))
        bound = [p for p in pods if (p.get("spec") or {}).get("nodeName")]
        if bound:
            try:      # the reference lists nodes from the API server, not a possibly lagging cache
                nodes = {n["metadata"]["name"] for n in (await self.client.list("nodes"))["items"]}
            except APIStatusError:
                nodes = None
            if nodes is not None:
                for p in bound:
                    if p["spec"]["nodeName"] not in nodes:
                        await self._force(p)
        for p in pods:
            if p["metadata"].get("deletionTimestamp") and not (p.get("spec") or {}).get("nodeName"):
                await self._force(p)

    async def _force(self, p):
        try:
            await self.client.delete("pods", p["metadata"]["name"], p["metadata"]["namespace"], grace_period=0)
        except APIStatusError as e:
            if not is_not_found(e):
                raise


from .nodelifecycle import NodeLifecycleController  # noqa: E402,F401  (re-export)
from .garbagecollector import GarbageCollector  # noqa: E402,F401  (re-export)
