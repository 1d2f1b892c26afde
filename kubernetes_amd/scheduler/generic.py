"""Generic scheduling algorithm: filter → extended-resource allocation → score → select.

Parity: `plugin/pkg/scheduler/core/generic_scheduler.go:109-365` (`Schedule`, `findNodesThatFit`
with the fork's `GetExtendedResources` call at :354-358, `PrioritizeNodes` :509, `selectHost`
round-robin among ties :177) and `algorithm.ScheduleAlgorithm.Schedule` returning
`(host, ExtendedResourceBinding)` (fork: scheduler_interface.go:49).

Differences by design:
  * predicates, the device allocation and scoring run in ONE pass per node (no separate
    Parallelize(16) fan-outs, no per-node deep copy of available devices);
  * a node that cannot possibly hold the pod's device count is rejected in O(1) before any
    predicate runs;
  * `percentage_of_nodes_to_score` (later-Kubernetes knob): stop filtering once enough feasible
    nodes are found, starting each cycle where the previous one stopped (fairness). 100 = the
    reference behaviour (score every node).
"""
from __future__ import annotations

import logging

from ..api import core
from . import predicates as P
from . import priorities as PR
from .cache import PodInfo, SchedulerCache
from .topology import POLICY_ANNOTATION, PREFERRED, Request, allocate

log = logging.getLogger("scheduler")


class FitError(Exception):
    def __init__(self, pod, num_nodes, failed: dict):
        self.pod = pod
        self.num_nodes = num_nodes
        self.failed = failed
        counts = {}
        for r in failed.values():
            counts[r] = counts.get(r, 0) + 1
        reasons = ", ".join(f"{n} {r}" for r, n in sorted(counts.items(), key=lambda kv: (-kv[1], kv[0])))
        super().__init__(f"0/{num_nodes} nodes are available: {reasons}.")


class CycleContext:
    """Per-pod scheduling-cycle state shared by predicates and priorities."""

    def __init__(self, cache: SchedulerCache, pod):
        self.cache = cache
        spec = pod.get("spec") or {}
        self.tolerates_unschedulable = any(
            t.get("key") == "node.kubernetes.io/unschedulable" and t.get("operator") == "Exists"
            for t in spec.get("tolerations") or ())
        ref = None
        for r in pod["metadata"].get("ownerReferences") or ():
            if r.get("controller"):
                ref = r.get("uid")
        self.owner_uid = ref
        self.node_affinity_prefs = PR.compile_node_affinity_prefs(pod)
        self.topo_scores = {}
        self.anti_affinity_terms = cache_anti_affinity(cache)
        self.any_anti_affinity = bool(self.anti_affinity_terms)

    def pods_by_topology(self, key, val):
        for ni in self.cache.nodes.values():
            if ni.labels.get(key) == val:
                for p, _ in ni.pods.values():
                    yield p

    def any_pod_matches(self, term, ns):
        for ni in self.cache.nodes.values():
            for p, _ in ni.pods.values():
                if P._pod_matches_term(p["metadata"].get("labels") or {}, p["metadata"].get("namespace"), term, ns):
                    return True
        return False

    def node_of(self, pod):
        st = self.cache.pod_states.get(f"{pod['metadata'].get('namespace')}/{pod['metadata']['name']}")
        return self.cache.nodes.get(st[1]) if st else None


def cache_anti_affinity(cache):
    out = []
    for p in cache.anti_pods.values():
        paa = (((p.get("spec") or {}).get("affinity") or {}).get("podAntiAffinity") or {})
        for t in paa.get("requiredDuringSchedulingIgnoredDuringExecution") or ():
            out.append((p, t))
    return out


class GenericScheduler:
    def __init__(self, cache: SchedulerCache, predicates=None, priorities=None, percentage_of_nodes_to_score=100,
                 extenders=None):
        self.cache = cache
        names = predicates or P.DEFAULT_PREDICATES
        self.predicates = [(n, P.PREDICATES[n]) for n in names]
        prios = priorities if priorities is not None else PR.DEFAULT_PRIORITIES
        self.priorities = [(n, w, *PR.PRIORITIES[n]) for n, w in prios.items() if w]
        self.pct = percentage_of_nodes_to_score
        self.extenders = extenders or []
        self._next_start = 0
        self._last_node_index = 0
        self._check_affinity = "MatchInterPodAffinity" in names

    def num_feasible_to_find(self, n):
        if self.pct >= 100 or n < 100:
            return n
        return max(100, n * self.pct // 100)

    def schedule(self, pod, pi: PodInfo | None = None):
        """Returns (node_name, extended_resource_binding)."""
        nodes = self.cache.node_list()
        if not nodes:
            raise FitError(pod, 0, {})
        pi = pi or PodInfo(pod)
        ctx = CycleContext(self.cache, pod) if (self._check_affinity or pi.er) else _LiteContext(self.cache, pod)
        policy = ((pod["metadata"].get("annotations") or {}).get(POLICY_ANNOTATION) or PREFERRED)
        reqs = [Request(name, rn, n, sel) for name, rn, n, sel in pi.er]
        need = {}
        for r in reqs:
            need[r.rname] = need.get(r.rname, 0) + r.count
        feasible, bindings, failed = [], {}, {}
        want = self.num_feasible_to_find(len(nodes))
        n = len(nodes)
        start = self._next_start % n
        preds = self.predicates
        checked = 0
        for off in range(n):
            ni = nodes[(start + off) % n]
            checked += 1
            reason = None
            for rn, cnt in need.items():
                if ni.er.free_count(rn) < cnt:
                    reason = f"Insufficient {rn}"
                    break
            if reason is None:
                for _, fn in preds:
                    reason = fn(pod, pi, ni, ctx)
                    if reason:
                        break
            if reason is None and reqs:
                binding, score, reason = allocate(reqs, ni.er, policy)
                if binding is not None:
                    bindings[ni.name] = binding
                    ctx.topo_scores[ni.name] = score
                    reason = reason or None
            if reason:
                failed[ni.name] = reason
                continue
            feasible.append(ni)
            if len(feasible) >= want:
                break
        self._next_start = start + checked
        for ext in self.extenders:
            feasible, efailed = ext.filter(pod, feasible)
            failed.update(efailed)
        if not feasible:
            raise FitError(pod, n, failed)
        if len(feasible) == 1:
            host = feasible[0].name
            return host, bindings.get(host, {})
        scores = self.prioritize(pod, pi, feasible, ctx)
        for ext in self.extenders:
            for name, s in ext.prioritize(pod, feasible).items():
                scores[name] = scores.get(name, 0) + s
        host = self.select_host(scores, feasible)
        return host, bindings.get(host, {})

    def prioritize(self, pod, pi, nodes, ctx):
        total = {ni.name: 0.0 for ni in nodes}
        for name, w, fn, reverse, norm in self.priorities:
            if name == "XGMITopologyPriority" and not pi.er:
                continue
            if name == "GPUBinPackingPriority" and not pi.er:
                continue
            if name == "SelectorSpreadPriority" and not ctx.owner_uid:
                continue
            if name == "NodeAffinityPriority" and not ctx.node_affinity_prefs:
                continue
            raw = [fn(pod, pi, ni, ctx) for ni in nodes]
            if norm:
                raw = PR.normalize(raw, reverse)
            for ni, s in zip(nodes, raw):
                total[ni.name] += w * s
        return total

    def select_host(self, scores, nodes):
        best = max(scores.values())
        ties = [ni.name for ni in nodes if scores[ni.name] == best]
        self._last_node_index += 1
        return ties[self._last_node_index % len(ties)]


class _LiteContext(CycleContext):
    """Context without the cluster-wide anti-affinity scan (no affinity predicate, no devices)."""

    def __init__(self, cache, pod):
        self.cache = cache
        spec = pod.get("spec") or {}
        self.tolerates_unschedulable = any(
            t.get("key") == "node.kubernetes.io/unschedulable" and t.get("operator") == "Exists"
            for t in spec.get("tolerations") or ())
        ref = None
        for r in pod["metadata"].get("ownerReferences") or ():
            if r.get("controller"):
                ref = r.get("uid")
        self.owner_uid = ref
        self.node_affinity_prefs = PR.compile_node_affinity_prefs(pod)
        self.topo_scores = {}
        self.anti_affinity_terms = []
        self.any_anti_affinity = False


def pod_is_gpu(pod) -> bool:
    return any(core.pod_extended_resource_name(per) == core.AMD_GPU
               for per in (pod.get("spec") or {}).get("extendedResources") or ())
