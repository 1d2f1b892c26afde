"""Generic scheduling algorithm: filter → extended-resource allocation → score → select.

Parity: `plugin/pkg/scheduler/core/generic_scheduler.go:109-365` (`Schedule`, `findNodesThatFit`
with the fork's `GetExtendedResources` call at :354-358, `PrioritizeNodes` :509, `selectHost`
round-robin among ties :177), `algorithm.ScheduleAlgorithm.Schedule` returning
`(host, ExtendedResourceBinding)` (fork: scheduler_interface.go:49), and the equivalence cache
(`plugin/pkg/scheduler/core/equivalence_cache.go`).

Differences by design:
  * predicates, the device-fit check and the raw priority values run in ONE pass per node;
    the device binding is materialised only for the selected node (no separate Parallelize(16)
    fan-outs, no per-node deep copy of available devices);
  * a node that cannot hold the pod's device count is rejected in O(1) (per-hive free counts);
  * equivalence cache: pods of one equivalence class (same resource/selector/toleration/device
    shape — e.g. every replica of a job, every density pod) reuse each node's evaluation
    until that node's generation changes. A bind touches one node, so the next pod of the
    class re-evaluates one node instead of all of them. Disabled for pods whose placement
    depends on other nodes' pods (inter-pod affinity) and when extenders are configured;
  * `percentage_of_nodes_to_score` (later-Kubernetes knob), default 100 = reference behaviour;
  * nominated pods (`podFitsOnNode` + `addNominatedPods`, generic_scheduler.go:367-486): a node
    with queued pods of equal or higher priority nominated to it (preemptors waiting for their
    victims to terminate) is checked twice — with those nominees accounted, including the device
    IDs they would take, and without — and bypasses the equivalence cache; the device binding
    comes from the first pass, so GPUs freed for a preemptor are never handed to a lower-priority
    pod. Nodes without such nominees take the usual path.
"""
from __future__ import annotations

import json
import logging
from collections import OrderedDict

from ..api import core
from . import predicates as P
from . import priorities as PR
from .cache import PodInfo, SchedulerCache
from .topology import POLICY_ANNOTATION, PREFERRED, Request, allocate, fast_path, feasible
from .whatif import WhatIfCache, nominated_view

log = logging.getLogger("scheduler")


class FitError(Exception):
    def __init__(self, pod, num_nodes, failed: dict):
        self.pod = pod
        self.num_nodes = num_nodes
        self.failed = failed
        counts = {}
        for rs in failed.values():
            for r in (rs if isinstance(rs, tuple) else (rs,)):
                counts[r] = counts.get(r, 0) + 1
        reasons = ", ".join(f"{n} {r}" for r, n in sorted(counts.items(), key=lambda kv: (-kv[1], kv[0])))
        super().__init__(f"0/{num_nodes} nodes are available: {reasons}.")


class CycleContext:
    """Per-pod scheduling-cycle state shared by predicates and priorities."""

    def __init__(self, cache: SchedulerCache, pod, with_affinity=True):
        self.cache = cache
        spec = pod.get("spec") or {}
        self.tolerates_unschedulable = any(
            t.get("key") == "node.kubernetes.io/unschedulable" and t.get("operator") == "Exists"
            for t in spec.get("tolerations") or ())
        ref = kind = None
        for r in pod["metadata"].get("ownerReferences") or ():
            if r.get("controller"):
                ref, kind = r.get("uid"), r.get("kind")
        self.owner_uid = ref
        self.owner_kind = kind
        self.node_affinity_prefs = PR.compile_node_affinity_prefs(pod)
        self.topo_scores = {}
        self.anti_affinity_terms = cache_anti_affinity(cache) if with_affinity else []
        self.any_anti_affinity = bool(self.anti_affinity_terms)
        self.volumes = cache.volumes
        self.pod = pod
        self.namespace = pod["metadata"].get("namespace", "default")
        self.affinity_prefs = _preferred_pod_affinity(pod)
        self._aff_counts = None
        self._svc = None
        self._svc_counts = {}
        self._svc_first = False

    # -- services selecting the pod (SelectorSpread, ServiceSpreading, ServiceAffinity, ...) ----
    @property
    def service_items(self):
        """[(service name, selector)] of the services in the pod's namespace that select it, by
        name (`GetPodServices`: a service without a selector selects nothing)."""
        if self._svc is None:
            svcs = self.cache.services.get(self.namespace)
            if not svcs:
                self._svc = ()
            else:
                labels = self.pod["metadata"].get("labels") or {}
                self._svc = [(n, sel) for n, sel in sorted(svcs.items())
                             if sel is not None and all(labels.get(k) == v for k, v in sel.items())]
        return self._svc

    @property
    def service_selectors(self):
        return [sel for _, sel in self.service_items]

    def service_label_counts(self, label):
        """({node label value: pods of the pod's first service there}, pods of that service)."""
        got = self._svc_counts.get(label)
        if got is None:
            counts, total = {}, 0
            items = self.service_items
            if items:
                sel = items[0][1]
                for pod, node in self.cache.pod_states.values():
                    if pod["metadata"].get("namespace", "default") != self.namespace:
                        continue
                    lbl = pod["metadata"].get("labels") or {}
                    if not all(lbl.get(k) == v for k, v in sel.items()):
                        continue
                    total += 1
                    ni = self.cache.nodes.get(node)
                    v = ni.labels.get(label) if ni is not None else None
                    if v is not None:
                        counts[v] = counts.get(v, 0) + 1
            got = self._svc_counts[label] = (counts, total)
        return got

    def service_affinity_first_node(self):
        """Node of the first placed pod whose labels carry this pod's labels (same namespace),
        when a service selects the pod (`serviceAffinityMetadataProducer`)."""
        if self._svc_first is False:
            self._svc_first = None
            if self.service_items:
                want = self.pod["metadata"].get("labels") or {}
                for pod, node in self.cache.pod_states.values():
                    if pod["metadata"].get("namespace", "default") != self.namespace or pod is self.pod:
                        continue
                    lbl = pod["metadata"].get("labels") or {}
                    if all(lbl.get(k) == v for k, v in want.items()):
                        self._svc_first = self.cache.nodes.get(node)
                        if self._svc_first is not None:
                            break
        return self._svc_first

    def pod_affinity_counts(self):
        """[(signed weight, topology key, {topology value: matching pods})] for the pod's
        preferred (anti-)affinity terms, computed once per cycle."""
        if self._aff_counts is None:
            out = []
            ns = self.pod["metadata"].get("namespace", "default")
            for w, term in self.affinity_prefs:
                key = term.get("topologyKey", "")
                if not key:
                    out.append((w, "", self._any_domain_counts(term, ns)))
                    continue
                counts = {}
                for ni in self.cache.nodes.values():
                    v = ni.labels.get(key)
                    if v is None:
                        continue
                    for p, _ in ni.pods.values():
                        if P._pod_matches_term(p["metadata"].get("labels") or {}, p["metadata"].get("namespace"), term, ns):
                            counts[v] = counts.get(v, 0) + 1
                out.append((w, key, counts))
            out += self._existing_pod_terms(ns)
            self._aff_counts = out
        return self._aff_counts

    def _shares_domain(self, a, b):
        for k in self.cache.failure_domains:
            v = a.labels.get(k)
            if v is not None and b.labels.get(k) == v:
                return True
        return False

    def _any_domain_counts(self, term, ns):
        """Empty topologyKey: {node name: matching pods on nodes sharing any failure domain}."""
        where = []
        for ni in self.cache.nodes.values():
            n = sum(1 for p, _ in ni.pods.values()
                    if P._pod_matches_term(p["metadata"].get("labels") or {}, p["metadata"].get("namespace"), term, ns))
            if n:
                where.append((ni, n))
        counts = {}
        if where:
            for ni in self.cache.nodes.values():
                c = sum(n for src, n in where if self._shares_domain(ni, src))
                if c:
                    counts[ni.name] = c
        return counts

    def _existing_pod_terms(self, ns):
        """Existing pods' terms that match the incoming pod (`interpod_affinity.go` symmetry):
        their required pod affinity scores `hard_pod_affinity_weight`, their preferred affinity
        +weight and preferred anti-affinity −weight, in their own topology domain."""
        cache = self.cache
        if not cache.affinity_pods:
            return []
        labels = self.pod["metadata"].get("labels") or {}
        hw = cache.hard_pod_affinity_weight
        out = []
        for key, p in cache.affinity_pods.items():
            st = cache.pod_states.get(key)
            ni = cache.nodes.get(st[1]) if st else None
            if ni is None:
                continue
            aff = (p.get("spec") or {}).get("affinity") or {}
            pns = p["metadata"].get("namespace", "default")
            terms = []
            pa = aff.get("podAffinity") or {}
            if hw:
                terms += [(float(hw), t) for t in pa.get("requiredDuringSchedulingIgnoredDuringExecution") or ()]
            terms += [(float(t.get("weight", 0)), t.get("podAffinityTerm") or {})
                      for t in pa.get("preferredDuringSchedulingIgnoredDuringExecution") or ()]
            terms += [(-float(t.get("weight", 0)), t.get("podAffinityTerm") or {})
                      for t in (aff.get("podAntiAffinity") or {}).get("preferredDuringSchedulingIgnoredDuringExecution") or ()]
            for w, term in terms:
                tkey = term.get("topologyKey", "")
                if not tkey:
                    if w and P._pod_matches_term(labels, ns, term, pns):
                        out.append((w, "", {o.name: 1 for o in cache.nodes.values() if self._shares_domain(o, ni)}))
                    continue
                v = ni.labels.get(tkey)
                if v is not None and w and P._pod_matches_term(labels, ns, term, pns):
                    out.append((w, tkey, {v: 1}))
        return out

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


def _preferred_pod_affinity(pod):
    aff = (pod.get("spec") or {}).get("affinity") or {}
    out = []
    for kind, sign in (("podAffinity", 1.0), ("podAntiAffinity", -1.0)):
        for wt in (aff.get(kind) or {}).get("preferredDuringSchedulingIgnoredDuringExecution") or ():
            out.append((sign * float(wt.get("weight", 0)), wt.get("podAffinityTerm") or {}))
    return out


def cache_anti_affinity(cache):
    out = []
    for p in cache.anti_pods.values():
        paa = (((p.get("spec") or {}).get("affinity") or {}).get("podAntiAffinity") or {})
        for t in paa.get("requiredDuringSchedulingIgnoredDuringExecution") or ():
            out.append((p, t))
    return out


def _has_pod_affinity(pod):
    aff = (pod.get("spec") or {}).get("affinity") or {}
    return bool(aff.get("podAffinity") or aff.get("podAntiAffinity"))


def equivalence_key(pod) -> str:
    """Everything predicates/priorities read from the pod, minus per-pod identity (names,
    UIDs, the ResourceV2-generated ER names)."""
    spec = pod.get("spec") or {}
    md = pod.get("metadata") or {}
    owner = None
    for r in md.get("ownerReferences") or ():
        if r.get("controller"):
            owner = r.get("uid")
    ers = [((per.get("resources") or {}).get("limits"), (per.get("affinity") or {}).get("required"))
           for per in spec.get("extendedResources") or ()]
    ctrs = [(c.get("resources"), [p.get("hostPort") for p in c.get("ports") or () if p.get("hostPort")])
            for c in (spec.get("containers") or []) + (spec.get("initContainers") or [])]
    proj = (md.get("namespace"), owner, spec.get("nodeName"), spec.get("nodeSelector"), spec.get("affinity"),
            spec.get("tolerations"), ers, ctrs, (md.get("annotations") or {}).get(POLICY_ANNOTATION))
    return json.dumps(proj, sort_keys=True, separators=(",", ":"))


class GenericScheduler:
    def __init__(self, cache: SchedulerCache, predicates=None, priorities=None, percentage_of_nodes_to_score=100,
                 extenders=None, equivalence_cache=True, ecache_classes=256):
        self.cache = cache
        # predicates: names from the registry, or (name, fn) for a Policy's argument-based
        # custom predicate; priorities: name -> weight, or name -> (weight, fn, reverse, normalize)
        self.predicates = [(n, P.PREDICATES[n]) if isinstance(n, str) else tuple(n)
                           for n in (predicates or P.DEFAULT_PREDICATES)]
        names = [n for n, _ in self.predicates]
        prios = priorities if priorities is not None else PR.DEFAULT_PRIORITIES
        self.priorities = []
        for n, w in prios.items():
            entry = (n, w, *PR.PRIORITIES[n]) if not isinstance(w, (tuple, list)) else (n, *w)
            if entry[1]:
                self.priorities.append(entry)
        # plugins whose answer for one node depends on pods on OTHER nodes (ServiceAffinity,
        # ServiceAntiAffinity): a node's cached evaluation would go stale, so no equivalence cache
        self.global_view = any(getattr(f, "global_view", False) for _, f in self.predicates) or \
            any(getattr(e[2], "global_view", False) for e in self.priorities)
        self.pct = percentage_of_nodes_to_score
        self.extenders = extenders or []
        self._next_start = 0
        self._last_node_index = 0
        self._check_affinity = "MatchInterPodAffinity" in names
        self.predicates_novol = [(n, f) for n, f in self.predicates if n not in P.VOLUME_PREDICATES]
        self.use_ecache = equivalence_cache
        self.ecache: OrderedDict[str, dict] = OrderedDict()
        self.ecache_classes = ecache_classes
        self.ecache_hits = 0
        self.ecache_misses = 0
        self.prefer = None   # node name -> bool: a scheduler shard's own nodes win among feasible ones
        self.queue = None    # SchedulingQueue: its nominated pods are accounted in the fit check

    def num_feasible_to_find(self, n):
        if self.pct >= 100 or n < 100:
            return n
        return max(100, n * self.pct // 100)

    def _active_priorities(self, pi, ctx):
        out = []
        for name, w, fn, reverse, norm in self.priorities:
            if name in ("XGMITopologyPriority", "GPUBinPackingPriority") and not pi.er:
                continue
            if name == "SelectorSpreadPriority" and not ctx.owner_uid and not ctx.service_items:
                continue
            if name == "ServiceSpreadingPriority" and not ctx.service_items:
                continue
            if name == "NodeAffinityPriority" and not ctx.node_affinity_prefs:
                continue
            if name == "InterPodAffinityPriority" and not ctx.affinity_prefs and not self.cache.affinity_pods:
                continue
            out.append((name, w, fn, reverse, norm))
        return out

    def schedule(self, pod, pi: PodInfo | None = None):
        """Returns (node_name, extended_resource_binding)."""
        nodes = self.cache.node_list()
        if not nodes:
            raise FitError(pod, 0, {})
        pi = pi or PodInfo(pod)
        affinity_sensitive = self._check_affinity and (_has_pod_affinity(pod) or bool(self.cache.anti_pods))
        ctx = CycleContext(self.cache, pod, with_affinity=affinity_sensitive)
        policy = ((pod["metadata"].get("annotations") or {}).get(POLICY_ANNOTATION) or PREFERRED)
        reqs = [Request(name, rn, n, sel) for name, rn, n, sel in pi.er]
        fast = bool(reqs) and fast_path(reqs)
        need = {}
        for r in reqs:
            need[r.rname] = need.get(r.rname, 0) + r.count
        prios = self._active_priorities(pi, ctx)
        ec = None
        if pi.volumes:
            preds_for_pod = self.predicates
        else:
            preds_for_pod = self.predicates_novol
        if self.use_ecache and not affinity_sensitive and not self.extenders and (fast or not reqs) \
                and not pi.volumes and not ctx.affinity_prefs and not self.global_view:
            key = equivalence_key(pod)
            if self.cache.services:
                # service-based spreading reads the pod's labels: the class includes its services
                key += "|svc:" + ",".join(n for n, _ in ctx.service_items)
            ec = self.ecache.get(key)
            if ec is None:
                ec = self.ecache[key] = {}
                if len(self.ecache) > self.ecache_classes:
                    self.ecache.popitem(last=False)
            else:
                self.ecache.move_to_end(key)
        fnodes, raws, bindings, failed = [], [], {}, {}
        want = self.num_feasible_to_find(len(nodes))
        n = len(nodes)
        start = self._next_start % n
        preds = preds_for_pod
        checked = 0
        hits = misses = 0
        # hot loop (every node, every pod): locals only; equivalence-cache failures are not
        # recorded per node here — FitError rebuilds the reasons on its (rare) path
        ec_get = ec.get if ec is not None else None
        ec_failed = [] if ec is not None else None
        topo = ctx.topo_scores
        f_append, r_append = fnodes.append, raws.append
        order = nodes[start:] + nodes[:start] if start else nodes
        nom = self.queue.nominated_pods if self.queue is not None else None
        for ni in order:
            checked += 1
            if nom:
                nominees = nom.get(ni.name)
                view = nominated_view(pod, ni, nominees) if nominees else None
                if view is not None:
                    vctx = CycleContext(WhatIfCache(self.cache, ni, view), pod, with_affinity=True) \
                        if affinity_sensitive else ctx
                    reason, score, binding = self._fit(pod, pi, view, vctx, preds, need, reqs, policy)
                    if reason is None:
                        reason = self._fit(pod, pi, ni, ctx, preds, need, reqs, policy)[0]
                    if reason:
                        failed[ni.name] = reason
                        continue
                    if binding is not None:
                        bindings[ni.name] = binding
                    if score is not None:
                        ctx.topo_scores[ni.name] = score
                    fnodes.append(ni)
                    raws.append(tuple(fn(pod, pi, ni, ctx) for _, _, fn, _, _ in prios))
                    if len(fnodes) >= want:
                        break
                    continue
            if ec_get is not None:
                ent = ec_get(ni.name)
                if ent is not None and ent[0] == ni.generation:
                    hits += 1
                    if ent[1]:
                        ec_failed.append(ni)
                        continue
                    topo[ni.name] = ent[2]
                    f_append(ni)
                    r_append(ent[3])
                    if len(fnodes) >= want:
                        break
                    continue
                misses += 1
            reason = None
            score = None
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
                if fast:
                    ok, score, reason = feasible(reqs, ni.er, policy)
                    if ok:
                        reason = None
                else:
                    binding, score, reason = allocate(reqs, ni.er, policy)
                    if binding is not None:
                        bindings[ni.name] = binding
                        reason = None
            raw = None
            if reason is None:
                if score is not None:
                    ctx.topo_scores[ni.name] = score
                raw = tuple(fn(pod, pi, ni, ctx) for _, _, fn, _, _ in prios)
            if ec is not None:
                ec[ni.name] = (ni.generation, reason, score, raw)
            if reason:
                failed[ni.name] = reason
                continue
            fnodes.append(ni)
            raws.append(raw)
            if len(fnodes) >= want:
                break
        self._next_start = start + checked
        self.ecache_hits += hits
        self.ecache_misses += misses
        for ext in self.extenders:
            keep, efailed = ext.filter(pod, fnodes)
            failed.update(efailed)
            keepset = {k.name for k in keep}
            raws = [r for f, r in zip(fnodes, raws) if f.name in keepset]
            fnodes = [f for f in fnodes if f.name in keepset]
        if not fnodes:
            for ni in ec_failed or ():
                failed[ni.name] = ec[ni.name][1]
            raise FitError(pod, n, failed)
        if self.prefer is not None and len(fnodes) > 1:
            own = [i for i, ni in enumerate(fnodes) if self.prefer(ni.name)]
            if own and len(own) < len(fnodes):
                fnodes = [fnodes[i] for i in own]
                raws = [raws[i] for i in own]
        if len(fnodes) == 1:
            host = fnodes[0].name
        else:
            scores = self._combine(prios, fnodes, raws)
            for ext in self.extenders:
                try:
                    escores = ext.prioritize(pod, fnodes)
                except Exception:   # generic_scheduler.go PrioritizeNodes: extender errors are ignored
                    log.warning("extender prioritize failed; ignoring its scores", exc_info=True)
                    continue
                for name, s in escores.items():
                    scores[name] = scores.get(name, 0) + s
            host = self.select_host(scores, fnodes)
        if host in bindings:
            return host, bindings[host]
        if fast:
            # materialise the device binding for the chosen node only
            binding, _, reason = allocate(reqs, self.cache.nodes[host].er, policy)
            if binding is None:  # cannot happen: feasible() and allocate() agree
                raise FitError(pod, n, {host: reason})
            return host, binding
        return host, {}

    @staticmethod
    def _fit(pod, pi, ni, ctx, preds, need, reqs, policy):
        """(reason, topology score, device binding) of one node, device binding materialised."""
        for rn, cnt in need.items():
            if ni.er.free_count(rn) < cnt:
                return f"Insufficient {rn}", None, None
        for _, fn in preds:
            reason = fn(pod, pi, ni, ctx)
            if reason:
                return reason, None, None
        if reqs:
            binding, score, reason = allocate(reqs, ni.er, policy)
            if binding is None:
                return reason, None, None
            return None, score, binding
        return None, None, None

    @staticmethod
    def _combine(prios, nodes, raws):
        total = [0.0] * len(nodes)
        for j, (_, w, _, reverse, norm) in enumerate(prios):
            col = [r[j] for r in raws]
            if norm == "minmax":
                col = PR.normalize_minmax(col)
            elif norm == "spread":
                col = PR.normalize_spread(col, nodes)
            elif callable(norm):          # a Policy / plugin reduce over the feasible nodes
                col = norm(col, nodes)
            elif norm:
                col = PR.normalize(col, reverse)
            for i, s in enumerate(col):
                total[i] += w * s
        return {ni.name: t for ni, t in zip(nodes, total)}

    def prioritize(self, pod, pi, nodes, ctx):
        prios = self._active_priorities(pi, ctx)
        raws = [tuple(fn(pod, pi, ni, ctx) for _, _, fn, _, _ in prios) for ni in nodes]
        return self._combine(prios, nodes, raws)

    def select_host(self, scores, nodes):
        best = max(scores.values())
        ties = [ni.name for ni in nodes if scores[ni.name] == best]
        self._last_node_index += 1
        return ties[self._last_node_index % len(ties)]


def pod_is_gpu(pod) -> bool:
    return any(core.pod_extended_resource_name(per) == core.AMD_GPU
               for per in (pod.get("spec") or {}).get("extendedResources") or ())
