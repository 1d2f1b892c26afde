"""Priority preemption, GPU-aware.

Parity with `plugin/pkg/scheduler/core/generic_scheduler.go`:
  * `Preempt` (:199-256): only after a FitError; `podEligibleToPreemptOthers` (:999-1011) — no
    second preemption while lower-priority pods on the preemptor's nominated node are still
    terminating; `nodesWherePreemptionMightHelp` (:957-991) — nodes that failed for a reason
    removing pods cannot fix are skipped, and when no node is left the preemptor's own
    nomination is cleared; the chosen node must pass the extenders with the victims removed
    (`nodePassesExtendersForPreemption`, :795-827), else the next-best node is tried; lower-
    priority pods nominated to the chosen node are returned for un-nomination
    (`getLowerPriorityNominatedPods`, :258-279).
  * `selectVictimsOnNode` (:883-953): remove every lower-priority pod, check the fit (with the
    equal/higher-priority nominees of the node added, `podFitsOnNode` + `addNominatedPods`
    :367-392), then reprieve — PDB-violating victims first, then the others, each group from
    the highest priority down (`filterPodsWithPDBViolation` :834-866).
  * `pickOneNodeForPreemption` (:663-756): fewest PDB violations, lowest highest-victim
    priority, smallest sum of (priority + 2^31), fewest victims, first.
  * the scheduler's side (`plugin/pkg/scheduler/scheduler.go:209-253`, factory podPreemptor
    `factory.go:1259-1300`): the `NominatedNodeName` ANNOTATION (generic_scheduler.go:66) is
    merge-patched through pods/status; victims are deleted; nominations of lower-priority pods
    are cleared by setting the annotation to "".

MI355X difference: victims free their *assigned devices*, so "does the preemptor fit" is the
full device allocator (hive/NUMA/attribute selectors) on a what-if copy of the node's device
accounting — removing two 1-GPU pods from different hives does not make room for a pod that
requires a fully connected 2-GPU set — and nominees hold real device IDs on the what-if copy
(`add_nominee`), so GPUs freed for a preemptor are not handed to a lower-priority pod created
during the victims' grace period.
"""
from __future__ import annotations

from ..api.labels import SelectorError, label_selector_as_selector
from ..api.meta import ns_name
from .generic import CycleContext
from .queue import NOMINATED_ANNOTATION, nominated_node_name
from .topology import POLICY_ANNOTATION, PREFERRED, Request, allocate
from .whatif import WhatIfCache, add_nominee, nominated_view

__all__ = ["NOMINATED_ANNOTATION", "nominated_node_name", "pod_priority", "preempt", "select_victims",
           "select_victims_on_node", "select_nodes_for_preemption", "pick_one_node_for_preemption",
           "nodes_where_preemption_might_help", "pod_eligible_to_preempt_others", "filter_pods_with_pdb_violation",
           "add_nominee", "nominated_view", "Victims"]

# predicate failures that removing pods from the node can never fix (generic_scheduler.go:968-979)
UNRESOLVABLE_REASONS = frozenset({
    "node(s) didn't match node selector",                          # ErrNodeSelectorNotMatch
    "node(s) didn't match the requested hostname",                 # ErrPodNotMatchHostName
    "node(s) had taints that the pod didn't tolerate",             # ErrTaintsTolerationsNotMatch
    "node(s) didn't have the requested labels",                    # ErrNodeLabelPresenceViolated
    "node(s) were not ready",                                      # ErrNodeNotReady
    "node(s) had unavailable network",                             # ErrNodeNetworkUnavailable
    "node(s) were unschedulable",                                  # ErrNodeUnschedulable
    "node(s) had unknown conditions",                              # ErrNodeUnknownCondition
    "node(s) had no available volume zone",                        # ErrVolumeZoneConflict
    "node(s) had volume node affinity conflict",                   # ErrVolumeNodeConflict
    "node(s) didn't find available persistent volumes to bind",    # ErrVolumeBindConflict
})

_PRIO_OFFSET = 2 ** 31      # math.MaxInt32 + 1 (pickOneNodeForPreemption :721)


def pod_priority(pod) -> int:
    return int((pod.get("spec") or {}).get("priority") or 0)


class Victims:
    """generic_scheduler.go:53-56."""
    __slots__ = ("pods", "num_pdb_violations")

    def __init__(self, pods, num_pdb_violations=0):
        self.pods = pods
        self.num_pdb_violations = num_pdb_violations

    def __repr__(self):
        return f"Victims({[p['metadata']['name'] for p in self.pods]}, pdb={self.num_pdb_violations})"


def _affinity_sensitive(gs, pod):
    if "MatchInterPodAffinity" not in {n for n, _ in gs.predicates}:
        return False
    aff = (pod.get("spec") or {}).get("affinity") or {}
    return bool(aff.get("podAffinity") or aff.get("podAntiAffinity") or gs.cache.anti_pods)


def node_fits(gs, pod, pi, ni, orig=None, nominees=None):
    """`podFitsOnNode` against one what-if NodeInfo: every predicate and the device allocator,
    first with the node's equal/higher-priority nominees added, then (if any were) without."""
    views = []
    view = nominated_view(pod, ni, nominees)
    if view is not None:
        views.append(view)
    views.append(ni)
    sensitive = _affinity_sensitive(gs, pod)
    need = {}
    for _, rn, n, _ in pi.er:
        need[rn] = need.get(rn, 0) + n
    for v in views:
        for rn, cnt in need.items():
            if v.er.free_count(rn) < cnt:
                return False
        cache = WhatIfCache(gs.cache, orig if orig is not None else gs.cache.nodes.get(ni.name, ni), v) \
            if sensitive else gs.cache
        ctx = CycleContext(cache, pod, with_affinity=sensitive)
        for _, fn in gs.predicates:
            if fn(pod, pi, v, ctx):
                return False
        if pi.er:
            policy = ((pod["metadata"].get("annotations") or {}).get(POLICY_ANNOTATION) or PREFERRED)
            binding, _, _ = allocate([Request(name, rn, n, sel) for name, rn, n, sel in pi.er], v.er, policy)
            if binding is None:
                return False
    return True


# -- PDBs -----------------------------------------------------------------------------------------

def filter_pods_with_pdb_violation(pods, pdbs):
    """(violating, non-violating), order preserved (generic_scheduler.go:834-866): a pod violates
    when a PDB of its namespace with a non-empty selector matching it allows no disruption."""
    violating, ok = [], []
    for p in pods:
        labels = p["metadata"].get("labels") or {}
        hit = False
        if labels:
            ns = p["metadata"].get("namespace", "default")
            for pdb in pdbs or ():
                if pdb["metadata"].get("namespace", "default") != ns:
                    continue
                try:
                    sel = label_selector_as_selector((pdb.get("spec") or {}).get("selector"))
                except SelectorError:
                    continue
                if sel.empty() or not sel.matches(labels):
                    continue
                st = pdb.get("status") or {}
                if int(st.get("disruptionsAllowed", st.get("podDisruptionsAllowed", 0)) or 0) <= 0:
                    hit = True
                    break
        (violating if hit else ok).append(p)
    return violating, ok


# -- victims --------------------------------------------------------------------------------------

def select_victims_on_node(gs, pod, pi, ni, pdbs=(), nominees=None):
    """(victims, number of PDB-violating victims, fits) — generic_scheduler.go:883-953."""
    prio = pod_priority(pod)
    sim = ni.clone()
    lower = []
    for k, (p, q) in list(ni.pods.items()):
        if pod_priority(p) < prio:
            lower.append((k, p, q))
            sim.remove_pod(k)
    # util.HigherPriorityPod order; the sort is stable, so equal priorities keep node order
    lower.sort(key=lambda t: -pod_priority(t[1]))
    if not node_fits(gs, pod, pi, sim, ni, nominees):
        return None, 0, False
    by_pod = {id(p): (k, p, q) for k, p, q in lower}
    violating, non_violating = filter_pods_with_pdb_violation([p for _, p, _ in lower], pdbs)
    victims = []
    n_violating = 0

    def reprieve(p):
        k, _, q = by_pod[id(p)]
        sim.add_pod(k, p, q)
        if node_fits(gs, pod, pi, sim, ni, nominees):
            return True
        sim.remove_pod(k)
        victims.append(p)
        return False

    for p in violating:
        if not reprieve(p):
            n_violating += 1
    for p in non_violating:
        reprieve(p)
    return victims, n_violating, True


def select_victims(gs, pod, pi, ni, pdbs=()):
    """Minimal set of lower-priority pods whose removal lets `pod` fit on `ni`, or None."""
    victims, _, fits = select_victims_on_node(gs, pod, pi, ni, pdbs)
    return victims if fits else None


def select_nodes_for_preemption(gs, pod, pi, nodes, pdbs=(), queue=None):
    """{node name: Victims} for every node where the pod fits after evictions (:760-793)."""
    out = {}
    for ni in nodes:
        nominees = queue.nominees_for_node(ni.name) if queue is not None else None
        victims, n_pdb, fits = select_victims_on_node(gs, pod, pi, ni, pdbs, nominees)
        if fits:
            out[ni.name] = Victims(victims, n_pdb)
    return out


def pick_one_node_for_preemption(node_victims):
    """generic_scheduler.go:663-756. `node_victims`: {node: Victims}, insertion-ordered."""
    if not node_victims:
        return None
    for n, v in node_victims.items():
        if not v.pods:
            return n          # a node that needs no preemption (pods terminated meanwhile)

    def narrow(cands, key):
        best = min(key(n) for n in cands)
        return [n for n in cands if key(n) == best]

    cands = list(node_victims)
    for key in (lambda n: node_victims[n].num_pdb_violations,
                lambda n: pod_priority(node_victims[n].pods[0]),
                lambda n: sum(pod_priority(p) + _PRIO_OFFSET for p in node_victims[n].pods),
                lambda n: len(node_victims[n].pods)):
        cands = narrow(cands, key)
        if len(cands) == 1:
            break
    return cands[0]


def pick_node(candidates):
    """Back-compat helper: {node: [victim pods]} -> node."""
    return pick_one_node_for_preemption({n: v if isinstance(v, Victims) else Victims(v) for n, v in candidates.items()})


def _reasons(r):
    if r is None:
        return ()
    return r if isinstance(r, (tuple, list)) else (r,)


def nodes_where_preemption_might_help(pod, nodes, failed):
    """generic_scheduler.go:957-991: nodes not failed for an unresolvable reason."""
    out = []
    for ni in nodes:
        name = ni if isinstance(ni, str) else ni.name
        if name not in failed or not any(r in UNRESOLVABLE_REASONS for r in _reasons(failed[name])):
            out.append(ni)
    return out


def pod_eligible_to_preempt_others(pod, cache):
    """generic_scheduler.go:999-1011: a pod already nominated to a node where lower-priority pods
    are still terminating (its earlier victims) must not preempt again."""
    name = nominated_node_name(pod)
    if name:
        ni = cache.nodes.get(name)
        if ni is not None:
            prio = pod_priority(pod)
            for p, _ in ni.pods.values():
                if p["metadata"].get("deletionTimestamp") and pod_priority(p) < prio:
                    return False
    return True


def node_passes_extenders(gs, pod, name, victims):
    """generic_scheduler.go:795-827 (HTTP extenders see node objects / names; the what-if
    removal only matters to in-process extenders, which receive the what-if NodeInfo)."""
    if not gs.extenders:
        return True, None
    ni = gs.cache.nodes[name]
    sim = ni.clone()
    for v in victims:
        sim.remove_pod(ns_name(v))
    nodes = [sim]
    for ext in gs.extenders:
        try:
            nodes, failed = ext.filter(pod, nodes)
        except Exception as e:  # noqa: BLE001 - an extender error rejects this node only
            return False, e
        if name in failed or not nodes:
            return False, None
    return True, None


def preempt(gs, pod, pi, fit_error=None, pdbs=(), queue=None):
    """`Preempt`: returns (node name | None, victims, pods whose nomination to clear).

    Without `fit_error` every node is a candidate (older callers)."""
    cache = gs.cache
    if not pod_eligible_to_preempt_others(pod, cache):
        return None, [], []
    prio = pod_priority(pod)
    if not any(pod_priority(p) < prio for p, _ in cache.pod_states.values()):
        return None, [], []     # nothing may be preempted anywhere: skip the per-node what-ifs
    all_nodes = [ni for ni in cache.node_list()]
    if not all_nodes:
        return None, [], []
    if fit_error is not None:
        potential = nodes_where_preemption_might_help(pod, all_nodes, fit_error.failed)
    else:
        potential = [ni for ni in all_nodes if ni.ready and not ni.unschedulable]
    if not potential:
        return None, [], [pod]
    node_victims = select_nodes_for_preemption(gs, pod, pi, potential, pdbs, queue)
    while node_victims:
        name = pick_one_node_for_preemption(node_victims)
        if name is None:
            break
        ok, _err = node_passes_extenders(gs, pod, name, node_victims[name].pods)
        if ok:
            clear = []
            if queue is not None:
                clear = [p for p, _ in queue.nominees_for_node(name).values()
                         if pod_priority(p) < prio and ns_name(p) != ns_name(pod)]
            return name, node_victims[name].pods, clear
        del node_victims[name]
    return None, [], []


def victim_keys(victims):
    return [ns_name(p) for p in victims]
