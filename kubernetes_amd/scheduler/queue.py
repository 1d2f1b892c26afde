"""Scheduling queue: active heap ordered by (priority desc, enqueue time), an unschedulable
set re-activated by cluster events, and per-pod exponential backoff.

Parity: `plugin/pkg/scheduler/core/scheduling_queue.go:49-738` (PriorityQueue: activeQ,
unschedulableQ, nominated pods, MoveAllToActiveQueue on node/pod events) and the
factory's backoff (`plugin/pkg/scheduler/factory/factory.go:1135-1180`, 1 s → 60 s).
"""
from __future__ import annotations

import asyncio
import heapq
import itertools
import time

from ..api.meta import ns_name
from .cache import PodInfo


class PodBackoff:
    def __init__(self, initial=1.0, maximum=60.0):
        self.initial, self.maximum = initial, maximum
        self.entries: dict[str, float] = {}

    def next(self, key):
        d = self.entries.get(key, self.initial / 2) * 2
        d = min(d, self.maximum)
        self.entries[key] = d
        return d

    def forget(self, key):
        self.entries.pop(key, None)


class SchedulingQueue:
    def __init__(self, unschedulable_flush=30.0):
        self._heap = []
        self._seq = itertools.count()
        self.active: dict[str, tuple] = {}      # key -> (pod, PodInfo, enqueue time)
        self.unschedulable: dict[str, tuple] = {}
        self.nominated: dict[str, str] = {}     # pod key -> node
        self.backoff = PodBackoff()
        self.conflict_backoff = PodBackoff(0.005, 0.5)   # lost bind races between scheduler shards
        self._ev = asyncio.Event()
        self._timers = {}
        self.unschedulable_flush = unschedulable_flush
        self._closed = False

    def __len__(self):
        return len(self.active)

    def _push(self, pod, pi=None, t=None):
        key = ns_name(pod)
        prio = int((pod.get("spec") or {}).get("priority") or 0)
        t = time.monotonic() if t is None else t
        self.active[key] = (pod, pi or PodInfo(pod), t)
        heapq.heappush(self._heap, (-prio, t, next(self._seq), key))
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
            self.active[key] = (new, PodInfo(new), t)
            return
        if key in self.unschedulable:
            if (old.get("spec") != new.get("spec")) or (old["metadata"].get("labels") != new["metadata"].get("labels")):
                del self.unschedulable[key]
                self._push(new)
            else:
                self.unschedulable[key] = (new, None, self.unschedulable[key][2])
            return
        if key not in self._timers:
            self._push(new)

    def delete(self, pod):
        key = ns_name(pod)
        self.active.pop(key, None)   # lazy removal from the heap
        self.unschedulable.pop(key, None)
        self.nominated.pop(key, None)
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

    def add_backoff(self, pod, conflict=False):
        """Re-queue after the pod's backoff (binding errors, API errors; `conflict`: a bind lost
        to another scheduler shard — short backoff, the winner's binding is already in flight)."""
        key = ns_name(pod)
        d = (self.conflict_backoff if conflict else self.backoff).next(key)
        self._cancel_timer(key)
        loop = asyncio.get_event_loop()
        self._timers[key] = loop.call_later(d, self._timer_fire, key, pod)

    def _timer_fire(self, key, pod):
        self._timers.pop(key, None)
        if key not in self.active:
            self._push(pod)

    def _cancel_timer(self, key):
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
