"""What-if views for preemption and nominated pods.

* `add_nominee` / `nominated_view` — `addNominatedPods`
  (`plugin/pkg/scheduler/core/generic_scheduler.go:367-392`): a clone of a NodeInfo with the
  node's nominated pods of equal or higher priority accounted, including device IDs.
* `WhatIfCache` — the scheduler cache with one node replaced by its what-if copy, so the
  cross-node predicates (inter-pod affinity) see victims removed / nominees added, as the
  reference's `meta.RemovePod` / `meta.AddPod` do (`selectVictimsOnNode`, :894-905).
"""
from __future__ import annotations

from ..api.meta import ns_name
from .cache import PodInfo
from .topology import POLICY_ANNOTATION, PREFERRED, Request, allocate


def pod_priority(pod) -> int:
    return int((pod.get("spec") or {}).get("priority") or 0)


def add_nominee(view, pod, pi=None):
    """Account a nominated (not yet bound) pod on `view`: its cpu/memory/ports like any pod, and
    — unlike the reference, whose scheduler cache has no per-device view of unbound pods —
    the device IDs the allocator would give it now, so they stay reserved. When the nominee does
    not fit yet (its victims still hold devices), every free device up to its count is held."""
    pi = pi or PodInfo(pod)
    if pi.er:
        assigned: dict[str, list] = {}
        policy = ((pod["metadata"].get("annotations") or {}).get(POLICY_ANNOTATION) or PREFERRED)
        binding, _, _ = allocate([Request(name, rn, n, sel) for name, rn, n, sel in pi.er], view.er, policy)
        if binding is not None:
            for name, rn, _, _ in pi.er:
                assigned.setdefault(rn, []).extend((binding.get(name) or {}).get("resources") or ())
        else:
            for _, rn, n, _ in pi.er:
                taken = set(assigned.get(rn, ()))
                free = [i for hf in (view.er.hive_free.get(rn) or {}).values() for i in hf if i not in taken]
                assigned.setdefault(rn, []).extend(free[:n])
        pi = pi.with_assigned(pod)
        pi.assigned = assigned
    view.add_pod(ns_name(pod), pod, pi)


def nominated_view(pod, ni, nominees):
    """`addNominatedPods` (generic_scheduler.go:367-392): a clone of `ni` with the nominees of
    equal or higher priority than `pod` added, or None when there is none (use `ni` as is)."""
    if not nominees:
        return None
    prio = pod_priority(pod)
    key = ns_name(pod)
    add = [(p, pi) for k, (p, pi) in nominees.items() if k != key and pod_priority(p) >= prio]
    if not add:
        return None
    view = ni.clone()
    for p, pi in add:
        add_nominee(view, p, pi)
    return view


# -- what-if view of the cache for inter-pod (anti-)affinity ------------------------------------

class _NodesOverlay:
    """`cache.nodes` with one NodeInfo replaced by its what-if copy."""
    __slots__ = ("base", "sim")

    def __init__(self, base, sim):
        self.base, self.sim = base, sim

    def get(self, name, default=None):
        return self.sim if name == self.sim.name else self.base.get(name, default)

    def __getitem__(self, name):
        return self.sim if name == self.sim.name else self.base[name]

    def __contains__(self, name):
        return name in self.base or name == self.sim.name

    def values(self):
        for ni in self.base.values():
            yield self.sim if ni.name == self.sim.name else ni

    def items(self):
        for name, ni in self.base.items():
            yield name, (self.sim if name == self.sim.name else ni)


class _PodStatesOverlay:
    __slots__ = ("base", "sim", "removed")

    def __init__(self, base, sim, removed):
        self.base, self.sim, self.removed = base, sim, removed

    def get(self, key, default=None):
        if key in self.removed:
            return default
        ent = self.sim.pods.get(key)
        if ent is not None:
            return (ent[0], self.sim.name)
        return self.base.get(key, default)

    def values(self):
        for key, st in self.base.items():
            if key not in self.removed and key not in self.sim.pods:
                yield st
        for p, _ in self.sim.pods.values():
            yield (p, self.sim.name)


class WhatIfCache:
    """The scheduler cache as seen with `sim` in place of its node (victims removed, nominees
    added), for the predicates that look across nodes (MatchInterPodAffinity)."""

    def __init__(self, cache, orig, sim):
        self._cache = cache
        removed = {k for k in orig.pods if k not in sim.pods}
        self.nodes = _NodesOverlay(cache.nodes, sim)
        self.pod_states = _PodStatesOverlay(cache.pod_states, sim, removed)
        anti = {k: p for k, p in cache.anti_pods.items() if k not in removed}
        aff = {k: p for k, p in cache.affinity_pods.items() if k not in removed}
        for k, (p, _) in sim.pods.items():
            a = (p.get("spec") or {}).get("affinity") or {}
            if ((a.get("podAntiAffinity") or {}).get("requiredDuringSchedulingIgnoredDuringExecution")):
                anti.setdefault(k, p)
            if a.get("podAffinity") or (a.get("podAntiAffinity") or {}).get("preferredDuringSchedulingIgnoredDuringExecution"):
                aff.setdefault(k, p)
        self.anti_pods, self.affinity_pods = anti, aff

    def __getattr__(self, name):       # services, volumes, failure_domains, ...
        return getattr(self._cache, name)
