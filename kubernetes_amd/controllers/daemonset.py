"""DaemonSet and StatefulSet controllers.

DaemonSet parity: `pkg/controller/daemon/daemon_controller.go` (nodeShouldRunDaemonPod: node
selector / affinity / taints-tolerations, one pod per eligible node, delete pods on nodes that
no longer qualify, status counts). Design choice: instead of the 1.9 behaviour of writing
`spec.nodeName` directly (`daemon_controller.go:1323` NewPod), each daemon pod is pinned with
required node affinity on the node's `kubernetes.io/hostname` label (the 1.9 NodeSelectorTerm
has no `matchFields`; the kubelet sets that label to the node name) and goes through the
scheduler — so a DaemonSet requesting `amd.com/gpu` (e.g. a per-node GPU burn-in / xGMI probe)
gets real device IDs allocated.

StatefulSet parity: `pkg/controller/statefulset/stateful_set_control.go` — ordinal pods
`<name>-<i>`, OrderedReady (create i only when 0..i-1 are Running and Ready, delete from the
highest ordinal) or Parallel pod management, RollingUpdate by revision hash in reverse
ordinal order, status replicas / readyReplicas / currentRevision / updateRevision.
"""
from __future__ import annotations

import asyncio

from ..api import meta as m
from ..client.rest import APIStatusError, is_already_exists, is_not_found
from ..scheduler import predicates as P
from ..scheduler.cache import NodeInfo, PodInfo
from .history import REVISION_HASH, ensure_revision, revisions_of
from .base import Controller, controller_ref, pod_from_template, pod_is_active, pod_is_ready, split_key

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
        ds = self.ds_inf.get(key)
        if ds is None or ds["metadata"].get("deletionTimestamp"):
            return
        ns, name = split_key(key)
        pods = [p for p in self.pod_inf.store.by_index("controllerUID", ds["metadata"]["uid"]) if pod_is_active(p)]
        by_node: dict[str, list] = {}
        for p in pods:
            by_node.setdefault(self._target_node(p), []).append(p)
        want = {n["metadata"]["name"] for n in self.node_inf.list() if node_should_run(ds, n)}
        creating = self._inflight.setdefault(key, set())
        creating &= want - set(by_node)
        tmpl = (ds.get("spec") or {}).get("template") or {}
        spec = ds.get("spec") or {}
        rev = await ensure_revision(self.client, ds, "DaemonSet", tmpl,
                                    revisions_of(self.rev_inf.list(), ds["metadata"]["uid"]),
                                    int(spec.get("revisionHistoryLimit", 10)))
        h = rev["metadata"]["labels"][REVISION_HASH]
        todo = [n for n in sorted(want) if n not in by_node and n not in creating]
        dels = [p for node, ps in by_node.items() if node not in want for p in ps]
        dels += [p for node, ps in by_node.items() if node in want for p in ps[1:]]
        # RollingUpdate (apps/v1 default): replace pods of older revisions, at most maxUnavailable
        # (default 1) nodes without a ready pod at a time; OnDelete waits for manual deletion
        strategy = spec.get("updateStrategy") or {}
        if strategy.get("type", "RollingUpdate") == "RollingUpdate" and not todo:
            max_unavail = int(((strategy.get("rollingUpdate") or {}).get("maxUnavailable")) or 1)
            unavailable = sum(1 for n in want if not any(pod_is_ready(p) for p in by_node.get(n, ())))
            stale = [ps[0] for node, ps in sorted(by_node.items()) if node in want and ps
                     and (ps[0]["metadata"].get("labels") or {}).get(REVISION_HASH) != h
                     and not ps[0]["metadata"].get("deletionTimestamp")]
            budget = max(0, max_unavail - unavailable)
            dels += [p for p in stale if not pod_is_ready(p)] + [p for p in stale if pod_is_ready(p)][:budget]

        async def create(node):
            pod = pod_from_template(tmpl, ds, f"{name}-", ns)
            pod["metadata"]["labels"][REVISION_HASH] = h
            spec = pod["spec"]
            spec["tolerations"] = list(spec.get("tolerations") or []) + DS_TOLERATIONS
            aff = spec.setdefault("affinity", {}).setdefault("nodeAffinity", {})
            aff["requiredDuringSchedulingIgnoredDuringExecution"] = {"nodeSelectorTerms": [
                {"matchExpressions": [{"key": HOSTNAME, "operator": "In", "values": [node]}]}]}
            creating.add(node)
            await self.client.create("pods", pod, ns)

        await asyncio.gather(*(create(n) for n in todo), return_exceptions=True)
        for p in dels:
            try:
                await self.client.delete("pods", p["metadata"]["name"], ns)
            except APIStatusError:
                pass
        ready = sum(1 for ps in by_node.values() for p in ps if pod_is_ready(p))
        st = {"desiredNumberScheduled": len(want), "currentNumberScheduled": len([n for n in by_node if n in want]),
              "numberMisscheduled": len([n for n in by_node if n not in want and n]), "numberReady": ready,
              "numberAvailable": ready,
              "updatedNumberScheduled": len([n for n, ps in by_node.items() if n in want and ps and
                                             (ps[0]["metadata"].get("labels") or {}).get(REVISION_HASH) == h]),
              "observedGeneration": ds["metadata"].get("generation", 1)}
        if {k: (ds.get("status") or {}).get(k) for k in st} != st:
            try:
                await self.client.patch("daemonsets", name, {"status": st}, ns, "merge", "status")
            except APIStatusError as e:
                if not is_not_found(e):
                    raise


from .statefulset import StatefulSetController  # noqa: E402,F401  (re-export)
