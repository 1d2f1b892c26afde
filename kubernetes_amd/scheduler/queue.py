"""Scheduling queue: active heap ordered by (priority desc, enqueue time), an unschedulable
set re-activated by cluster events, and per-pod exponential backoff.

Parity: `plugin/pkg/scheduler/core/scheduling_queue.go:49-738` (PriorityQueue: activeQ,
unschedulableQ, MoveAllToActiveQueue on node/pod events) and the factory's backoff
(`plugin/pkg/scheduler/factory/factory.go:1135-1180`, 1 s → 60 s).

Nominated pods (`scheduling_queue.go:134-234,456-466`): every queued pod — active, unschedulable
or waiting out a backoff — whose `NominatedNodeName` annotation names a node is indexed under
that node; `nominees_for_node` is `WaitingPodsForNode`. A pod leaves the index while it is being
scheduled (`Pop`) and comes back if it is requeued, so it never competes with its own
nomination.
"""
from __future__ import annotations

import asyncio
import heapq
import itertools
import time

from ..api.meta import ns_name
from .cache import PodInfo

# generic_scheduler.go:66 NominatedNodeAnnotationKey
NOMINATED_ANNOTATION = "NominatedNodeName"


def nominated_node_name(pod) -> str:
    """scheduling_queue.go:134-141 (an empty value = no nomination: the reference clears it
    by writing "")."""
    return ((pod.get("metadata") or {}).get("annotations") or {}).get(NOMINATED_ANNOTATION) or ""


class PodBackoff:
    """`plugin/pkg/scheduler/util/backoff_utils.go` PodBackoff: per-pod exponential backoff
    (initial, doubling, capped at maximum); entries untouched for longer than the maximum are
    garbage-collected (`Gc`, also run every 1024 updates), so a pod seen again later starts over."""

    def __init__(self, initial=1.0, maximum=60.0, clock=time.monotonic):
        self.initial, self.maximum = initial, maximum
        self.clock = clock
        self.entries: dict[str, float] = {}
        self.updated: dict[str, float] = {}
        self._ops = 0

    def next(self, key):
        d = self.entries.get(key, self.initial / 2) * 2
        d = min(d, self.maximum)
        self.entries[key] = d
        self.updated[key] = self.clock()
        self._ops += 1
        if self._ops & 1023 == 0:
            self.gc()
        return d

    def forget(self, key):
        self.entries.pop(key, None)
        self.updated.pop(key, None)

    def gc(self):
        now = self.clock()
        for key in [k for k, t in self.updated.items() if now - t > self.maximum]:
            self.forget(key)


class SchedulingQueue:
    def __init__(self, unschedulable_flush=30.0):
        self._heap = []
        self._seq = itertools.count()
        self.active: dict[str, tuple] = {}      # key -> (pod, PodInfo, enqueue time)
        self.unschedulable: dict[str, tuple] = {}
        self.nominated: dict[str, str] = {}     # pod key -> nominated node
        self.nominated_pods: dict[str, dict[str, tuple]] = {}   # node -> {pod key: (pod, PodInfo)}
        self.backoff = PodBackoff()
        self.conflict_backoff = PodBackoff(0.005, 0.5)   # lost bind races between scheduler shards
        self._ev = asyncio.Event()
        self._timers = {}
        self._backoff_pods: dict[str, dict] = {}     # latest object of a pod waiting out a backoff
        self._aff_unsched: dict[str, dict] = {}       # unschedulable pods with required pod affinity (lazy)
        self.unschedulable_flush = unschedulable_flush
        self._closed = False

    def __len__(self):
        return len(self.active)

    # -- nominated pods --------------------------------------------------------------
    def _add_nominated(self, pod, pi=None):
        node = nominated_node_name(pod)
        key = ns_name(pod)
        if self.nominated.get(key) not in (None, node):
            self._delete_nominated(key)
        if not node:
            return
        self.nominated[key] = node
        self.nominated_pods.setdefault(node, {})[key] = (pod, pi or PodInfo(pod))

    def _delete_nominated(self, key):
        node = self.nominated.pop(key, None)
        if node is None:
            return
        d = self.nominated_pods.get(node)
        if d is not None:
            d.pop(key, None)
            if not d:
                del self.nominated_pods[node]

    def nominate(self, pod, node):
        """Record (node) or clear ("") a pod's nomination at once, ahead of the informer's copy
        of the annotated pod; the queued object is replaced by the annotated copy."""
        key = ns_name(pod)
        md = dict(pod["metadata"])
        md["annotations"] = dict(md.get("annotations") or {}, **{NOMINATED_ANNOTATION: node})
        new = dict(pod, metadata=md)
        if key in self.unschedulable:
            ent = self.unschedulable[key]
            self.unschedulable[key] = (new, ent[1], ent[2])
        elif key in self.active:
            ent = self.active[key]
            self.active[key] = (new, ent[1], ent[2])
        elif key in self._backoff_pods:
            self._backoff_pods[key] = new
        else:
            self._delete_nominated(key)
            return
        self._add_nominated(new)

    def nominees_for_node(self, node) -> dict:
        """`WaitingPodsForNode`: {pod key: (pod, PodInfo)} nominated to `node`."""
        return self.nominated_pods.get(node) or {}

    def waiting_pods_for_node(self, node) -> list:
        return [p for p, _ in self.nominees_for_node(node).values()]

    def _push(self, pod, pi=None, t=None):
        key = ns_name(pod)
        prio = int((pod.get("spec") or {}).get("priority") or 0)
        t = time.monotonic() if t is None else t
        pi = pi or PodInfo(pod)
        self.active[key] = (pod, pi, t)
        heapq.heappush(self._heap, (-prio, t, next(self._seq), key))
        if key in self.nominated or nominated_node_name(pod):
            self._add_nominated(pod, pi)
        self._ev.set()

    def add(self, pod):
        key = ns_name(pod)
        self.unschedulable.pop(key, None)
        self._cancel_timer(key)
        self._push(pod)

    def update(self, old, new):
        key = ns_name(new)
        if key in self.active:
            _, _, t = self.active[key]
            pi = PodInfo(new)
            self.active[key] = (new, pi, t)
            self._add_nominated(new, pi)
            return
        if key in self.unschedulable:
            self._add_nominated(new)
            if (old.get("spec") != new.get("spec")) or (old["metadata"].get("labels") != new["metadata"].get("labels")):
                del self.unschedulable[key]
                self._push(new)
            else:
                self.unschedulable[key] = (new, None, self.unschedulable[key][2])
            return
        if key in self._timers:
            self._backoff_pods[key] = new
            self._add_nominated(new)     # waiting out a backoff: still a queued pod
        else:
            self._push(new)

    def delete(self, pod):
        key = ns_name(pod)
        self.active.pop(key, None)   # lazy removal from the heap
        self.unschedulable.pop(key, None)
        self._delete_nominated(key)
        self._cancel_timer(key)
        self.backoff.forget(key)
        self.conflict_backoff.forget(key)

    def unschedulable_pods(self):
        return [ent[0] for ent in self.unschedulable.values()]

    def unschedulable_since(self):
        """(pod, monotonic time it was marked unschedulable)."""
        return [(ent[0], ent[2]) for ent in self.unschedulable.values()]

    def add_unschedulable(self, pod):
        key = ns_name(pod)
        if key in self.active:
            return
        self.unschedulable[key] = (pod, None, time.monotonic())
        self._add_nominated(pod)
        if ((((pod.get("spec") or {}).get("affinity") or {}).get("podAffinity") or {})
                .get("requiredDuringSchedulingIgnoredDuringExecution")):
            self._aff_unsched[key] = pod

    def assigned_pod_added(self, pod):
        """`AssignedPodAdded` / `AssignedPodUpdated` (scheduling_queue.go:387-454): a bound pod
        whose labels match a required pod-affinity term of an unschedulable pod makes that pod
        schedulable again — move it to the active queue now rather than at the next flush."""
        if not self._aff_unsched:
            return
        from .predicates import _pod_matches_term
        md = pod.get("metadata") or {}
        labels, pns = md.get("labels") or {}, md.get("namespace", "default")
        for key, up in list(self._aff_unsched.items()):
            ent = self.unschedulable.get(key)
            if ent is None:
                del self._aff_unsched[key]
                continue
            up = ent[0]
            ns = up["metadata"].get("namespace", "default")
            terms = ((((up.get("spec") or {}).get("affinity") or {}).get("podAffinity") or {})
                     .get("requiredDuringSchedulingIgnoredDuringExecution") or ())
            if any(_pod_matches_term(labels, pns, t, ns) for t in terms):
                del self.unschedulable[key]
                del self._aff_unsched[key]
                self._push(up)

    def add_backoff(self, pod, conflict=False):
        """Re-queue after the pod's backoff (binding errors, API errors; `conflict`: a bind lost
        to another scheduler shard — short backoff, the winner's binding is already in flight)."""
        key = ns_name(pod)
        d = (self.conflict_backoff if conflict else self.backoff).next(key)
        self._cancel_timer(key)
        self._add_nominated(pod)
        self._backoff_pods[key] = pod
        loop = asyncio.get_event_loop()
        self._timers[key] = loop.call_later(d, self._timer_fire, key, pod)

    def _timer_fire(self, key, pod):
        self._timers.pop(key, None)
        pod = self._backoff_pods.pop(key, pod)
        if key not in self.active:
            self._push(pod)

    def _cancel_timer(self, key):
        self._backoff_pods.pop(key, None)
        h = self._timers.pop(key, None)
        if h is not None:
            h.cancel()

    def move_all_to_active(self):
        if not self.unschedulable:
            return
        for key, (pod, _, _) in list(self.unschedulable.items()):
            self._push(pod)
        self.unschedulable.clear()

    def flush_unschedulable_leftover(self):
        now = time.monotonic()
        for key, (pod, _, t) in list(self.unschedulable.items()):
            if now - t > self.unschedulable_flush:
                del self.unschedulable[key]
                self._push(pod)

    def pop_nowait(self):
        while self._heap:
            _, t, _, key = heapq.heappop(self._heap)
            ent = self.active.get(key)
            if ent is None or ent[2] != t:
                continue  # stale heap entry
            del self.active[key]
            if self.nominated:
                self._delete_nominated(key)   # PriorityQueue.Pop: not its own competitor
            return ent
        return None

    async def pop(self):
        while True:
            ent = self.pop_nowait()
            if ent is not None:
                return ent
            if self._closed:
                return None
            self._ev.clear()
            await self._ev.wait()

    def close(self):
        self._closed = True
        self._ev.set()
        for h in self._timers.values():
            h.cancel()
        self._timers.clear()
