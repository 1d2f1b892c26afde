"""Priority preemption, GPU-aware.

Parity: `plugin/pkg/scheduler/core/generic_scheduler.go:199-265` (`Preempt`),
`:663-1011` (`selectNodesForPreemption`, `selectVictimsOnNode` with the remove-all-lower then
reprieve-highest-first loop, `pickOneNodeForPreemption`: lowest highest-victim priority, then
smallest priority sum, then fewest victims) and the scheduler's use at
`plugin/pkg/scheduler/scheduler.go:207-250` (nominatedNodeName on the preemptor, delete victims).

MI355X difference: victims free their *assigned devices*, so "does the preemptor fit" is the
full device allocator (hive/NUMA/attribute selectors) on a what-if copy of the node's device
accounting — removing two 1-GPU pods from different hives does not make room for a pod that
requires a fully connected 2-GPU set.
"""
from __future__ import annotations

from ..api.meta import ns_name
from .generic import CycleContext
from .topology import POLICY_ANNOTATION, PREFERRED, Request, allocate


def pod_priority(pod) -> int:
    return int((pod.get("spec") or {}).get("priority") or 0)


def node_fits(gs, pod, pi, ni) -> bool:
    """Every predicate and the device allocator against one (what-if) NodeInfo."""
    need = {}
    for _, rn, n, _ in pi.er:
        need[rn] = need.get(rn, 0) + n
    for rn, cnt in need.items():
        if ni.er.free_count(rn) < cnt:
            return False
    ctx = CycleContext(gs.cache, pod, with_affinity=False)
    for _, fn in gs.predicates:
        if fn(pod, pi, ni, ctx):
            return False
    if pi.er:
        policy = ((pod["metadata"].get("annotations") or {}).get(POLICY_ANNOTATION) or PREFERRED)
        binding, _, _ = allocate([Request(name, rn, n, sel) for name, rn, n, sel in pi.er], ni.er, policy)
        return binding is not None
    return True


def select_victims(gs, pod, pi, ni):
    """Minimal set of lower-priority pods whose removal lets `pod` fit on `ni`, or None."""
    prio = pod_priority(pod)
    lower = [(k, p, q) for k, (p, q) in ni.pods.items() if pod_priority(p) < prio]
    if not lower:
        return None
    sim = ni.clone()
    for k, _, _ in lower:
        sim.remove_pod(k)
    if not node_fits(gs, pod, pi, sim):
        return None
    # reprieve as many as possible, highest priority first
    victims = []
    for k, p, q in sorted(lower, key=lambda t: -pod_priority(t[1])):
        sim.add_pod(k, p, q)
        if not node_fits(gs, pod, pi, sim):
            sim.remove_pod(k)
            victims.append(p)
    return victims


def pick_node(candidates):
    """candidates: {node: [victim pods]} -> node (generic_scheduler.go pickOneNodeForPreemption)."""
    if not candidates:
        return None
    for n, v in candidates.items():
        if not v:
            return n          # fits without victims (a race with a deletion): take it
    return min(candidates, key=lambda n: (max(pod_priority(p) for p in candidates[n]),
                                          sum(pod_priority(p) for p in candidates[n]),
                                          len(candidates[n]), n))


def preempt(gs, pod, pi):
    """Returns (node name, victims) or (None, []) if preemption cannot help."""
    if pod_priority(pod) <= 0 and not any(pod_priority(p) < 0 for ni in gs.cache.node_list() for p, _ in ni.pods.values()):
        return None, []
    cands = {}
    for ni in gs.cache.node_list():
        if not ni.ready or ni.unschedulable:
            continue
        v = select_victims(gs, pod, pi, ni)
        if v is not None:
            cands[ni.name] = v
    node = pick_node(cands)
    if node is None:
        return None, []
    return node, cands[node]


def victim_keys(victims):
    return [ns_name(p) for p in victims]
