"""DaemonSet controller.

Parity: `pkg/controller/daemon/daemon_controller.go` — `nodeShouldRunDaemonPod` (:1239) with its
three answers (wantToRun / shouldSchedule / shouldContinueRunning) from a simulation of the
GeneralPredicates and taints against the node's other pods (`simulate` :1153): a node selector,
host-name or host-port miss means "not here at all"; an untolerated NoSchedule taint keeps running
pods but places none; an untolerated NoExecute taint evicts; insufficient resources keep running
pods, place none and raise FailedPlacement, and the set is parked as "suspended" on that node
until a pod there is deleted (`requeueSuspendedDaemonPods` :562). `manage` (:808): one pod per
node, failed pods deleted (the sync then errors, so the rate limiter paces kill/recreate loops),
duplicates beyond the oldest deleted; pods claimed through the ControllerRefManager (adopt
orphans, release non-matching); creates in slow-start batches of at most burstReplicas.
`updateDaemonSetStatus` (:1027) counts over each node's oldest pod, numberAvailable honouring
minReadySeconds. Node updates re-sync only when labels, taints or true conditions change AND the
answer changes (`updateNode` :699). `update.go`: RollingUpdate — every old unavailable pod goes at
once, old available pods go while fewer than maxUnavailable (int or percentage of the desired
count, rounded up: `getUnavailableNumbers` :386-422) nodes are unavailable; ControllerRevision
history with `cleanupHistory`.

Design choice: instead of the 1.9 behaviour of writing `spec.nodeName` directly
(`daemon_controller.go:1323` NewPod), each daemon pod is pinned with required node affinity on the
node's `kubernetes.io/hostname` label (the 1.9 NodeSelectorTerm has no `matchFields`; the kubelet
sets that label to the node name) and goes through the scheduler — so a DaemonSet requesting
`amd.com/gpu` (e.g. a per-node GPU burn-in / xGMI probe) gets real device IDs allocated.
"""
from __future__ import annotations

import asyncio

from ..api import core
from ..api import meta as m
from ..api.labels import SelectorError, label_selector_as_selector
from ..client.rest import APIStatusError, is_not_found
from ..scheduler import predicates as P
from ..scheduler.cache import NodeInfo, PodInfo
from .deployment_util import value_from_int_or_percent
from .history import REVISION_HASH, ensure_revision, revisions_of, truncate_history
from .base import (Controller, claim_objects, controller_ref, pod_from_template, pod_is_available, pod_is_ready,
                   split_key)

HOSTNAME = "kubernetes.io/hostname"
TEMPLATE_GENERATION = "pod-template-generation"
BURST_REPLICAS = 250            # `daemon_controller.go` BurstReplicas
FAILED_PLACEMENT = "FailedPlacement"

# `util.CreatePodTemplate` / `simulate`: daemon pods survive taint-based eviction of not-ready and
# unreachable nodes and tolerate the node-pressure NoSchedule taints; the unschedulable toleration
# lets this framework's scheduler place them on cordoned nodes, as the 1.9 controller (which
# bypassed the scheduler) did.
DS_TOLERATIONS = [
    {"key": "node.kubernetes.io/not-ready", "operator": "Exists", "effect": "NoExecute"},
    {"key": "node.kubernetes.io/unreachable", "operator": "Exists", "effect": "NoExecute"},
    {"key": "node.kubernetes.io/disk-pressure", "operator": "Exists", "effect": "NoSchedule"},
    {"key": "node.kubernetes.io/memory-pressure", "operator": "Exists", "effect": "NoSchedule"},
    {"key": "node.kubernetes.io/unschedulable", "operator": "Exists", "effect": "NoSchedule"},
]


class _Ctx:
    tolerates_unschedulable = True


OUT_OF_DISK_TOLERATION = {"key": "node.kubernetes.io/out-of-disk", "operator": "Exists", "effect": "NoExecute"}
CRITICAL_POD_ANNOTATION = "scheduler.alpha.kubernetes.io/critical-pod"     # kubelettypes.CriticalPodAnnotationKey


def _with_tolerations(spec, meta=None):
    """CreatePodTemplate's tolerations (`AddOrUpdateTolerationInPodSpec`: a toleration with the
    same key and effect is replaced); a critical daemon pod (ExperimentalCriticalPodAnnotation,
    kube-system + empty critical-pod annotation) also tolerates the out-of-disk NoExecute taint."""
    tols = [dict(t) for t in spec.get("tolerations") or []]
    want = list(DS_TOLERATIONS)
    md = meta or {}
    from ..utils.features import DefaultFeatureGate
    if DefaultFeatureGate("ExperimentalCriticalPodAnnotation") and md.get("namespace") == "kube-system" and \
            (md.get("annotations") or {}).get(CRITICAL_POD_ANNOTATION) == "":
        want.append(OUT_OF_DISK_TOLERATION)
    for t in want:
        same = [i for i, x in enumerate(tols) if x.get("key") == t["key"] and x.get("effect") == t["effect"]]
        if same:
            tols[same[0]] = dict(t)
        else:
            tols.append(dict(t))
    return tols


def _tolerates_no_execute(pod, node):
    tols = (pod.get("spec") or {}).get("tolerations") or []
    return all(core.tolerates(tols, t) for t in (node.get("spec") or {}).get("taints") or ()
               if t.get("effect") == core.TAINT_NO_EXECUTE)


def node_should_run(ds, node, node_pods=()):
    """`nodeShouldRunDaemonPod` -> (wantToRun, shouldSchedule, shouldContinueRunning, reason):
    `node_pods` are the node's other pods (terminal ones and this set's own are ignored);
    `reason` is the FailedPlacement message when the pod wants to run but cannot be placed."""
    tmpl = (ds.get("spec") or {}).get("template") or {}
    tspec = tmpl.get("spec") or {}
    name = node["metadata"]["name"]
    if tspec.get("nodeName") and tspec["nodeName"] != name:
        return False, False, False, None
    spec = m.fast_copy(tspec)
    spec["nodeName"] = name
    spec["tolerations"] = _with_tolerations(spec, {"namespace": ds["metadata"].get("namespace"),
                                                   "annotations": (tmpl.get("metadata") or {}).get("annotations")})
    pod = {"metadata": {"name": "probe", "namespace": ds["metadata"].get("namespace"),
                        "labels": dict((tmpl.get("metadata") or {}).get("labels") or {})}, "spec": spec}
    ni = NodeInfo()
    ni.set_node(node)
    uid = ds["metadata"].get("uid")
    for p in node_pods:
        if (p.get("status") or {}).get("phase") in ("Succeeded", "Failed"):
            continue
        ref = controller_ref(p)
        if ref and ref.get("uid") == uid:
            continue
        ni.add_pod(m.ns_name(p), p, PodInfo(p))
    pi, ctx = PodInfo(pod), _Ctx()
    # intentional on the operator's part: not this node at all
    if P.match_node_selector(pod, pi, ni, ctx) or P.pod_fits_host_ports(pod, pi, ni, ctx):
        return False, False, False, None
    want = sched = cont = True
    if P.pod_tolerates_node_taints(pod, pi, ni, ctx):
        if not _tolerates_no_execute(pod, node):
            return False, False, False, None
        want = sched = False
    short = P.pod_fits_resources(pod, pi, ni, ctx)
    if isinstance(short, tuple):
        short = ", ".join(short)
    if sched and short:
        return want, False, cont, f"failed to place pod on {name!r}: {short}"
    return want, sched, cont, None


def node_in_same_condition(old, cur):
    """`nodeInSameCondition`: the same set of condition types are True."""
    return {c.get("type") for c in old or () if c.get("status") == "True"} == \
        {c.get("type") for c in cur or () if c.get("status") == "True"}


def is_pod_updated(generation, pod, h):
    """`util.IsPodUpdated`: the revision hash label matches, or (older pods) the template
    generation label."""
    labels = pod["metadata"].get("labels") or {}
    return (bool(h) and labels.get(REVISION_HASH) == h) or labels.get(TEMPLATE_GENERATION) == str(generation)


class DaemonSetController(Controller):
    name = "daemonset"

    def setup(self):
        self.ds_inf = self.factory.get("daemonsets")
        self.node_inf = self.factory.get("nodes")
        self.pod_inf = self.factory.get("pods")
        self.ds_inf.add_handler(self.enqueue, lambda o, n: self.enqueue(n), self.enqueue)
        self.node_inf.add_handler(self._add_node, self._update_node, None)
        self.pod_inf.add_handler(self._add_pod, self._update_pod, self._delete_pod_event)
        store = self.pod_inf.store
        if "controllerUID" not in store.indexers:
            store.add_indexer("controllerUID", lambda p: [r["uid"] for r in (p["metadata"].get("ownerReferences") or ()) if r.get("controller")])
        if "namespace" not in store.indexers:
            store.add_indexer("namespace", lambda p: [p["metadata"].get("namespace", "")])
        if "nodeName" not in store.indexers:
            store.add_indexer("nodeName", lambda p: [(p.get("spec") or {}).get("nodeName", "")])
        self.rev_inf = self.factory.get("controllerrevisions")
        self._inflight: dict[str, set] = {}
        self.suspended: dict[str, set] = {}        # node -> DaemonSet keys that want to run but cannot

    # -- event handlers ------------------------------------------------------------------------
    def _node_pods(self, name):
        return [p for p in self.pod_inf.store.by_index("nodeName", name) if (p.get("spec") or {}).get("nodeName") == name]

    def _add_node(self, node):
        """`addNode`: sets that should schedule onto the new node."""
        for ds in self.ds_inf.list():
            if node_should_run(ds, node, self._node_pods(node["metadata"]["name"]))[1]:
                self.enqueue(ds)

    def _update_node(self, old, cur):
        """`updateNode`: ignore updates that keep labels, taints and true conditions; otherwise
        re-sync the sets whose shouldSchedule / shouldContinueRunning answer changed."""
        if (old["metadata"].get("labels") or {}) == (cur["metadata"].get("labels") or {}) and \
                ((old.get("spec") or {}).get("taints") or []) == ((cur.get("spec") or {}).get("taints") or []) and \
                node_in_same_condition((old.get("status") or {}).get("conditions"),
                                       (cur.get("status") or {}).get("conditions")):
            return
        pods = self._node_pods(cur["metadata"]["name"])
        for ds in self.ds_inf.list():
            _, s0, c0, _ = node_should_run(ds, old, pods)
            _, s1, c1, _ = node_should_run(ds, cur, pods)
            if (s0, c0) != (s1, c1):
                self.enqueue(ds)

    def _resolve(self, pod, ref):
        if not ref or ref.get("kind") != "DaemonSet":
            return None
        ds = self.ds_inf.get(f"{pod['metadata'].get('namespace')}/{ref.get('name')}")
        return ds if ds is not None and ds["metadata"].get("uid") == ref.get("uid") else None

    def _sets_for_orphan(self, pod):
        out = []
        labels = pod["metadata"].get("labels") or {}
        for ds in self.ds_inf.list():
            if ds["metadata"].get("namespace") != pod["metadata"].get("namespace"):
                continue
            try:
                sel = label_selector_as_selector((ds.get("spec") or {}).get("selector"))
            except SelectorError:
                continue
            if not sel.empty() and sel.matches(labels):
                out.append(ds)
        return out

    def _add_pod(self, pod):
        if pod["metadata"].get("deletionTimestamp"):
            self._delete_pod_event(pod)
            return
        ref = controller_ref(pod)
        if ref is not None:
            ds = self._resolve(pod, ref)
            if ds is not None:
                self.enqueue(ds)
            return
        for ds in self._sets_for_orphan(pod):
            self.enqueue(ds)

    def _update_pod(self, old, cur):
        if old["metadata"].get("resourceVersion") == cur["metadata"].get("resourceVersion"):
            return
        oref, cref = controller_ref(old), controller_ref(cur)
        if oref != cref and oref is not None:
            ds = self._resolve(old, oref)
            if ds is not None:
                self.enqueue(ds)
        if cref is not None:
            ds = self._resolve(cur, cref)
            if ds is None:
                return
            self.enqueue(ds)
            mrs = int((ds.get("spec") or {}).get("minReadySeconds") or 0)
            if mrs and not pod_is_ready(old) and pod_is_ready(cur):
                self.queue.add_after(m.ns_name(ds), float(mrs) + 1.0)
            return
        if (old["metadata"].get("labels") or {}) != (cur["metadata"].get("labels") or {}) or oref != cref:
            for ds in self._sets_for_orphan(cur):
                self.enqueue(ds)

    def _delete_pod_event(self, pod):
        """`deletePod`: a daemon pod's set re-syncs; any other scheduled pod frees room, so the
        sets suspended on its node re-sync (rate limited)."""
        ds = self._resolve(pod, controller_ref(pod))
        if ds is not None:
            self.enqueue(ds)
            return
        node = (pod.get("spec") or {}).get("nodeName")
        if node:
            for key in list(self.suspended.get(node, ())):
                if self.ds_inf.get(key) is not None:
                    self.queue.add_rate_limited(key)

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

    # -- sync ----------------------------------------------------------------------------------
    async def sync(self, key):
        """`syncDaemonSet` (daemon_controller.go:1082): history, manage, rolling update, history
        cleanup, status."""
        ds = self.ds_inf.get(key)
        if ds is None:
            self._inflight.pop(key, None)
            for sets in self.suspended.values():
                sets.discard(key)
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
        if ds["metadata"].get("deletionTimestamp"):
            await self.update_status(ds, h)
            return
        by_node = await self.nodes_to_daemon_pods(ds)
        failed = await self.manage(ds, key, by_node, h)
        if (spec.get("updateStrategy") or {}).get("type", "RollingUpdate") == "RollingUpdate":
            want = {n["metadata"]["name"] for n in self.node_inf.list()
                    if node_should_run(ds, n, self._node_pods(n["metadata"]["name"]))[0]}
            await self.rolling_update(ds, want, await self.nodes_to_daemon_pods(ds, claim=False), h)
        live = {m.name_of(rev)} | {r["metadata"]["name"] for r in revisions
                                   if (r["metadata"].get("labels") or {}).get(REVISION_HASH) in
                                   {(p["metadata"].get("labels") or {}).get(REVISION_HASH)
                                    for ps in by_node.values() for p in ps}}
        await truncate_history(self.client, revisions, live, int(spec.get("revisionHistoryLimit", 10)))
        await self.update_status(ds, h)
        if failed:
            # `manage`: an error so the rate limiter paces a kill-recreate hot loop
            raise RuntimeError(f"deleted {failed} failed pods of DaemonSet {key}")

    async def nodes_to_daemon_pods(self, ds, claim=True):
        """`getNodesToDaemonPods`: the set's pods (claimed through the ControllerRefManager:
        matching orphans adopted, owned pods whose labels stopped matching released) by node,
        oldest first."""
        uid = ds["metadata"]["uid"]
        if claim:
            try:
                sel = label_selector_as_selector((ds.get("spec") or {}).get("selector"))
            except SelectorError:
                return {}
            pods = await claim_objects(self.client, ds, "pods",
                                       self.pod_inf.store.by_index("namespace", ds["metadata"].get("namespace", "")),
                                       lambda p: sel.matches(p["metadata"].get("labels") or {}))
        else:
            pods = self.pod_inf.store.by_index("controllerUID", uid)
        out: dict[str, list] = {}
        for p in pods:
            out.setdefault(self._target_node(p), []).append(p)
        for ps in out.values():
            ps.sort(key=lambda p: (m.parse_rfc3339(p["metadata"].get("creationTimestamp")) or 0, m.name_of(p)))
        return out

    async def manage(self, ds, key, by_node, h):
        """`manage` (:808): returns the number of failed pods deleted."""
        ns, name = split_key(key)
        creating = self._inflight.setdefault(key, set())
        creating -= {n for n, ps in by_node.items() if any(not _terminating(p) for p in ps)}
        todo, dels, failed = [], [], 0
        for node in self.node_inf.list():
            nname = node["metadata"]["name"]
            want, sched, cont, reason = node_should_run(ds, node, self._node_pods(nname))
            pods = by_node.get(nname, [])
            self.suspended.get(nname, set()).discard(key)
            if want and not sched:
                self.suspended.setdefault(nname, set()).add(key)
                creating.discard(nname)
                if reason:
                    self.recorder.event(ds, "Warning", FAILED_PLACEMENT, reason)
            elif sched and not pods:
                if nname not in creating:
                    todo.append(nname)
            elif cont:
                running = []
                for p in pods:
                    if _terminating(p):
                        continue
                    if (p.get("status") or {}).get("phase") == "Failed":
                        self.recorder.event(ds, "Warning", "FailedDaemonPod",
                                            f"Found failed daemon pod {ns}/{m.name_of(p)} on node {nname}, will try to kill it")
                        dels.append(p)
                        failed += 1
                    else:
                        running.append(p)
                dels += running[1:]
            elif pods:
                creating.discard(nname)
                dels += pods
            if not self.suspended.get(nname, True):
                del self.suspended[nname]
        todo, dels = todo[:BURST_REPLICAS], dels[:BURST_REPLICAS]
        tmpl = (ds.get("spec") or {}).get("template") or {}
        generation = (ds.get("spec") or {}).get("templateGeneration")

        async def create(node):
            pod = pod_from_template(tmpl, ds, f"{name}-", ns)
            pod["metadata"]["labels"][REVISION_HASH] = h
            if generation is not None:
                pod["metadata"]["labels"][TEMPLATE_GENERATION] = str(generation)
            spec = pod["spec"]
            spec["tolerations"] = _with_tolerations(spec, pod["metadata"])
            aff = spec.setdefault("affinity", {}).setdefault("nodeAffinity", {})
            aff["requiredDuringSchedulingIgnoredDuringExecution"] = {"nodeSelectorTerms": [
                {"matchExpressions": [{"key": HOSTNAME, "operator": "In", "values": [node]}]}]}
            creating.add(node)
            try:
                await self.client.create("pods", pod, ns)
            except APIStatusError:
                creating.discard(node)
                raise

        # slow start (`syncNodes` :923): batches of 1, 2, 4, ... stop at the first failing batch
        errs, pos, batch = [], 0, 1
        while pos < len(todo):
            res = await asyncio.gather(*(create(n) for n in todo[pos:pos + batch]), return_exceptions=True)
            bad = [r for r in res if isinstance(r, Exception)]
            errs += bad
            pos += batch
            if bad:
                break
            batch *= 2
        await asyncio.gather(*(self._delete_pod(p) for p in dels))
        if errs:
            self.recorder.event(ds, "Warning", "FailedCreate", f"Error creating: {errs[0]}")
            raise errs[0]
        return failed

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

    async def update_status(self, ds, h):
        """`updateDaemonSetStatus` (:1027): over every node, desired = wantToRun; counts over
        each node's oldest pod; numberAvailable honours minReadySeconds; written with the
        status subresource (`storeDaemonSetStatus`, conflict -> re-read and retry)."""
        spec = ds.get("spec") or {}
        mrs = int(spec.get("minReadySeconds") or 0)
        generation = spec.get("templateGeneration")
        by_node = await self.nodes_to_daemon_pods(ds, claim=False)
        desired = current = mis = ready = updated = available = 0
        for node in self.node_inf.list():
            nname = node["metadata"]["name"]
            pods = by_node.get(nname) or []
            if node_should_run(ds, node, self._node_pods(nname))[0]:
                desired += 1
                if pods:
                    current += 1
                    pod = pods[0]
                    if pod_is_ready(pod):
                        ready += 1
                        if pod_is_available(pod, mrs):
                            available += 1
                    if is_pod_updated(generation, pod, h):
                        updated += 1
            elif pods:
                mis += 1
        st = {"desiredNumberScheduled": desired, "currentNumberScheduled": current, "numberMisscheduled": mis,
              "numberReady": ready, "numberAvailable": available, "numberUnavailable": desired - available,
              "updatedNumberScheduled": updated}
        gen = ds["metadata"].get("generation", 1)
        if mrs and ready != available:
            self.queue.add_after(m.ns_name(ds), float(mrs))
        cur = ds.get("status") or {}
        if {k: cur.get(k, 0) for k in st} == st and cur.get("observedGeneration", 0) >= gen:
            return
        obj = ds
        for _ in range(3):        # StatusUpdateRetries
            upd = dict(obj)
            upd["status"] = dict(obj.get("status") or {}, observedGeneration=gen, **st)
            try:
                await self.client.update_status("daemonsets", upd, m.namespace_of(ds))
                return
            except APIStatusError as e:
                if is_not_found(e):
                    return
                if e.code != 409:
                    raise
            obj = await self.client.get("daemonsets", m.name_of(ds), m.namespace_of(ds))


def _terminating(p):
    return bool(p["metadata"].get("deletionTimestamp"))


from .statefulset import StatefulSetController  # noqa: E402,F401  (re-export)
