"""DaemonSet controller.

Parity: `pkg/controller/daemon/daemon_controller.go` (nodeShouldRunDaemonPod: node selector /
affinity / taints-tolerations; `manage`: one pod per eligible node, failed pods replaced,
duplicates and pods on nodes that no longer qualify deleted; `updateDaemonSetStatus`: counts over
each node's oldest pod, numberAvailable honouring minReadySeconds) and `update.go` (RollingUpdate:
every old unavailable pod goes at once, old available pods go while fewer than maxUnavailable —
an int or a percentage of the desired count, rounded up (`getUnavailableNumbers`, `:386-422`) —
nodes are unavailable; ControllerRevision history with `cleanupHistory`).

Design choice: instead of the 1.9 behaviour of writing `spec.nodeName` directly
(`daemon_controller.go:1323` NewPod), each daemon pod is pinned with required node affinity on the
node's `kubernetes.io/hostname` label (the 1.9 NodeSelectorTerm has no `matchFields`; the kubelet
sets that label to the node name) and goes through the scheduler — so a DaemonSet requesting
`amd.com/gpu` (e.g. a per-node GPU burn-in / xGMI probe) gets real device IDs allocated.
"""
from __future__ import annotations

import asyncio

from ..api import meta as m
from ..client.rest import APIStatusError, is_already_exists, is_not_found
from ..scheduler import predicates as P
from ..scheduler.cache import NodeInfo, PodInfo
from .deployment_util import value_from_int_or_percent
from .history import REVISION_HASH, ensure_revision, revisions_of, truncate_history
from .base import Controller, controller_ref, pod_from_template, pod_is_available, pod_is_ready, split_key

HOSTNAME = "kubernetes.io/hostname"

DS_TOLERATIONS = [
    {"key": "node.kubernetes.io/not-ready", "operator": "Exists", "effect": "NoExecute"},
    {"key": "node.kubernetes.io/unreachable", "operator": "Exists", "effect": "NoExecute"},
    {"key": "node.kubernetes.io/unschedulable", "operator": "Exists", "effect": "NoSchedule"},
]


class _Ctx:
    tolerates_unschedulable = True


def node_should_run(ds, node) -> bool:
    tmpl = (ds.get("spec") or {}).get("template") or {}
    pod = {"metadata": {"name": "probe", "namespace": ds["metadata"]["namespace"]},
           "spec": m.fast_copy(tmpl.get("spec") or {})}
    pod["spec"]["tolerations"] = list(pod["spec"].get("tolerations") or []) + DS_TOLERATIONS
    ni = NodeInfo()
    ni.set_node(node)
    pi = PodInfo(pod)
    for fn in (P.match_node_selector, P.pod_tolerates_node_taints):
        if fn(pod, pi, ni, _Ctx()):
            return False
    return True


class DaemonSetController(Controller):
    name = "daemonset"

    def setup(self):
        self.ds_inf = self.factory.get("daemonsets")
        self.node_inf = self.factory.get("nodes")
        self.pod_inf = self.factory.get("pods")
        self.ds_inf.add_handler(self.enqueue, lambda o, n: self.enqueue(n), None)
        self.node_inf.add_handler(self._all, lambda o, n: self._all(n), self._all)
        self.pod_inf.add_handler(self._pod, lambda o, n: self._pod(n), self._pod)
        if "controllerUID" not in self.pod_inf.store.indexers:
            self.pod_inf.store.add_indexer("controllerUID", lambda p: [r["uid"] for r in (p["metadata"].get("ownerReferences") or ()) if r.get("controller")])
        self.rev_inf = self.factory.get("controllerrevisions")
        self._inflight: dict[str, set] = {}

    def _all(self, _obj):
        for ds in self.ds_inf.list():
            self.enqueue(ds)

    def _pod(self, pod):
        ref = controller_ref(pod)
        if ref and ref.get("kind") == "DaemonSet":
            self.enqueue(f"{pod['metadata']['namespace']}/{ref['name']}")

    @staticmethod
    def _target_node(pod):
        nn = (pod.get("spec") or {}).get("nodeName")
        if nn:
            return nn
        aff = ((pod.get("spec") or {}).get("affinity") or {}).get("nodeAffinity") or {}
        for t in (aff.get("requiredDuringSchedulingIgnoredDuringExecution") or {}).get("nodeSelectorTerms") or ():
            for f in t.get("matchExpressions") or ():
                if f.get("key") == HOSTNAME and f.get("operator") == "In" and f.get("values"):
                    return f["values"][0]
        return None

    async def sync(self, key):
        """`syncDaemonSet` (daemon_controller.go:1090): history, manage, rolling update, history
        cleanup, status."""
        ds = self.ds_inf.get(key)
        if ds is None:
            return
        sel = (ds.get("spec") or {}).get("selector") or {}
        if not (sel.get("matchLabels") or sel.get("matchExpressions")):
            self.recorder.event(ds, "Warning", "SelectingAll",
                                "This daemon set is selecting all pods. A non-empty selector is required.")
            return
        spec = ds.get("spec") or {}
        tmpl = spec.get("template") or {}
        revisions = revisions_of(self.rev_inf.list(), ds["metadata"]["uid"])
        rev = await ensure_revision(self.client, ds, "DaemonSet", tmpl, revisions, limit=None)
        h = rev["metadata"]["labels"][REVISION_HASH]
        nodes = self.node_inf.list()
        want = {n["metadata"]["name"] for n in nodes if node_should_run(ds, n)}
        by_node = self.nodes_to_daemon_pods(ds)
        if not ds["metadata"].get("deletionTimestamp"):
            await self.manage(ds, key, want, by_node, h)
            if (spec.get("updateStrategy") or {}).get("type", "RollingUpdate") == "RollingUpdate":
                await self.rolling_update(ds, want, self.nodes_to_daemon_pods(ds), h)
            live = {m.name_of(rev)} | {r["metadata"]["name"] for r in revisions
                                       if (r["metadata"].get("labels") or {}).get(REVISION_HASH) in
                                       {(p["metadata"].get("labels") or {}).get(REVISION_HASH)
                                        for ps in by_node.values() for p in ps}}
            await truncate_history(self.client, revisions, live, int(spec.get("revisionHistoryLimit", 10)))
        await self.update_status(ds, want, self.nodes_to_daemon_pods(ds), h)

    def nodes_to_daemon_pods(self, ds):
        out: dict[str, list] = {}
        for p in self.pod_inf.store.by_index("controllerUID", ds["metadata"]["uid"]):
            if p["metadata"].get("deletionTimestamp") and (p.get("status") or {}).get("phase") in ("Failed", "Succeeded"):
                continue
            out.setdefault(self._target_node(p), []).append(p)
        for ps in out.values():
            ps.sort(key=lambda p: (m.parse_rfc3339(p["metadata"].get("creationTimestamp")) or 0, m.name_of(p)))
        return out

    async def manage(self, ds, key, want, by_node, h):
        """`manage` / `podsShouldBeOnNode`: one pod per eligible node; failed pods are replaced;
        duplicates (all but the oldest) and pods on ineligible nodes are deleted."""
        ns, name = split_key(key)
        creating = self._inflight.setdefault(key, set())
        creating &= want - {n for n, ps in by_node.items() if any(not _terminating(p) for p in ps)}
        todo, dels = [], []
        for node in sorted(want):
            pods = by_node.get(node, [])
            running = []
            for p in pods:
                if _terminating(p):
                    continue
                if (p.get("status") or {}).get("phase") == "Failed":
                    self.recorder.event(ds, "Warning", "FailedDaemonPod",
                                        f"Found failed daemon pod {ns}/{m.name_of(p)} on node {node}, will try to kill it")
                    dels.append(p)
                else:
                    running.append(p)
            if not running and node not in creating:
                todo.append(node)
            dels += running[1:]
        dels += [p for node, ps in by_node.items() if node not in want for p in ps if not _terminating(p)]
        tmpl = (ds.get("spec") or {}).get("template") or {}

        async def create(node):
            pod = pod_from_template(tmpl, ds, f"{name}-", ns)
            pod["metadata"]["labels"][REVISION_HASH] = h
            spec = pod["spec"]
            spec["tolerations"] = list(spec.get("tolerations") or []) + DS_TOLERATIONS
            aff = spec.setdefault("affinity", {}).setdefault("nodeAffinity", {})
            aff["requiredDuringSchedulingIgnoredDuringExecution"] = {"nodeSelectorTerms": [
                {"matchExpressions": [{"key": HOSTNAME, "operator": "In", "values": [node]}]}]}
            creating.add(node)
            try:
                await self.client.create("pods", pod, ns)
            except APIStatusError:
                creating.discard(node)
                raise
        res = await asyncio.gather(*(create(n) for n in todo), return_exceptions=True)
        for p in dels:
            await self._delete_pod(p)
        errs = [r for r in res if isinstance(r, Exception)]
        if errs:
            self.recorder.event(ds, "Warning", "FailedCreate", f"Error creating: {errs[0]}")
            raise errs[0]

    async def _delete_pod(self, p):
        try:
            await self.client.delete("pods", m.name_of(p), m.namespace_of(p))
        except APIStatusError as e:
            if not is_not_found(e):
                raise

    def unavailable_numbers(self, ds, want, by_node):
        """`getUnavailableNumbers` (update.go:386): (maxUnavailable resolved against the desired
        count, rounding up; nodes without an available, non-terminating pod)."""
        mrs = int((ds.get("spec") or {}).get("minReadySeconds") or 0)
        unavailable = 0
        for node in want:
            if not any(pod_is_available(p, mrs) and not _terminating(p) for p in by_node.get(node, ())):
                unavailable += 1
        mu = (((ds.get("spec") or {}).get("updateStrategy") or {}).get("rollingUpdate") or {}).get("maxUnavailable", 1)
        return value_from_int_or_percent(mu, len(want), True), unavailable

    async def rolling_update(self, ds, want, by_node, h):
        """`rollingUpdate` (update.go:44): delete every old unavailable pod, then old available
        pods while fewer than maxUnavailable nodes are unavailable."""
        mrs = int((ds.get("spec") or {}).get("minReadySeconds") or 0)
        old = [p for ps in by_node.values() for p in ps
               if (p["metadata"].get("labels") or {}).get(REVISION_HASH) != h]
        max_unavail, num_unavail = self.unavailable_numbers(ds, want, by_node)
        dels = [p for p in old if not pod_is_available(p, mrs) and not _terminating(p)]
        for p in old:
            if not pod_is_available(p, mrs) or _terminating(p):
                continue
            if num_unavail >= max_unavail:
                break
            dels.append(p)
            num_unavail += 1
        for p in dels:
            await self._delete_pod(p)
        return [m.name_of(p) for p in dels]

    async def update_status(self, ds, want, by_node, h):
        """`updateDaemonSetStatus` (daemon_controller.go:1025): counts over each node's oldest
        pod; numberAvailable honours minReadySeconds."""
        mrs = int((ds.get("spec") or {}).get("minReadySeconds") or 0)
        desired = current = mis = ready = updated = available = 0
        nodes = {n["metadata"]["name"] for n in self.node_inf.list()}
        for node in nodes | set(want):
            pods = by_node.get(node) or []
            if node in want:
                desired += 1
                if pods:
                    current += 1
                    pod = pods[0]
                    if pod_is_ready(pod):
                        ready += 1
                        if pod_is_available(pod, mrs):
                            available += 1
                    if (pod["metadata"].get("labels") or {}).get(REVISION_HASH) == h:
                        updated += 1
            elif pods:
                mis += 1
        st = {"desiredNumberScheduled": desired, "currentNumberScheduled": current, "numberMisscheduled": mis,
              "numberReady": ready, "numberAvailable": available, "numberUnavailable": desired - available,
              "updatedNumberScheduled": updated, "observedGeneration": ds["metadata"].get("generation", 1)}
        if mrs and ready != available:
            self.queue.add_after(m.ns_name(ds), float(mrs))
        if {k: (ds.get("status") or {}).get(k, 0) for k in st} != st:
            try:
                await self.client.patch("daemonsets", m.name_of(ds), {"status": st}, m.namespace_of(ds),
                                        "merge", "status")
            except APIStatusError as e:
                if not is_not_found(e):
                    raise


def _terminating(p):
    return bool(p["metadata"].get("deletionTimestamp"))


from .statefulset import StatefulSetController  # noqa: E402,F401  (re-export)
