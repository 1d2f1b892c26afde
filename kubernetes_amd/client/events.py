"""Event recorder. Parity: `staging/src/k8s.io/client-go/tools/record` (EventRecorder,
broadcaster → sink, aggregation of repeated events by incrementing `count`).

Events are queued and written by a small async worker pool so the caller's hot loop
(scheduleOne, pod sync) never waits on the API server. Like the reference, delivery is best
effort and bounded: an optional QPS/burst limit on event writes (the kubelet's
`--event-qps=5 --event-burst=10`, `pkg/kubelet/apis/kubeletconfig` EventRecordQPS/EventBurst,
applied to its event client) and a bounded queue (`record.maxQueuedEvents` = 1000) past which
new events are dropped rather than slowing the component down.
"""
from __future__ import annotations

import asyncio
import logging
import time

from ..api.meta import new_uid, now_rfc3339

log = logging.getLogger("events")


class EventRecorder:
    def __init__(self, client, component: str, host: str = "", workers: int = 4, max_queue: int = 1000,
                 enabled: bool = True, qps: float = 0.0, burst: int = 0):
        self.client = client
        self.source = {"component": component}
        if host:
            self.source["host"] = host
        self.enabled = enabled
        self.q: asyncio.Queue = asyncio.Queue(max_queue)
        self._workers = []
        self._n = workers
        self.sent = 0
        self.dropped = 0
        self._agg: dict[tuple, dict] = {}   # (involved uid, reason, message) -> last event
        self.qps, self.burst = qps, max(1, burst or int(qps) or 1)
        self._tokens = float(self.burst)
        self._last = time.monotonic()
        self.emitted: list = []             # for tests: (type, reason, message)

    def start(self):
        if self.enabled and not self._workers:
            self._workers = [asyncio.ensure_future(self._work()) for _ in range(self._n)]

    def stop(self):
        for w in self._workers:
            w.cancel()
        self._workers = []

    def event(self, obj, etype: str, reason: str, message: str, field_path: str = ""):
        self.emitted.append((etype, reason, message))
        if len(self.emitted) > 1000:
            del self.emitted[:500]
        if not self.enabled:
            return
        if self.q.full():
            # the bounded queue drops new events (record.maxQueuedEvents); do not build them
            self.dropped += 1
            return
        md = obj.get("metadata") or {}
        ns = md.get("namespace") or "default"
        key = (md.get("uid"), field_path, reason, message)
        now = now_rfc3339()
        prev = self._agg.get(key)
        if prev is not None and time.time() - prev["_t"] < 600:
            prev["count"] += 1
            prev["lastTimestamp"] = now
            prev["_t"] = time.time()
            ev = {k: v for k, v in prev.items() if k != "_t"}
            ev["_update"] = True
        else:
            ev = {"apiVersion": "v1", "kind": "Event",
                  "metadata": {"name": f"{md.get('name', 'unknown')}.{new_uid()[:16]}", "namespace": ns},
                  "involvedObject": {"kind": obj.get("kind", ""), "namespace": md.get("namespace", ""),
                                     "name": md.get("name", ""), "uid": md.get("uid", ""),
                                     "apiVersion": obj.get("apiVersion", "v1"),
                                     "resourceVersion": md.get("resourceVersion", ""),
                                     **({"fieldPath": field_path} if field_path else {})},
                  "reason": reason, "message": message, "type": etype, "source": self.source,
                  "firstTimestamp": now, "lastTimestamp": now, "count": 1}
            self._agg[key] = dict(ev, _t=time.time())
            if len(self._agg) > 4096:
                for k in list(self._agg)[:2048]:
                    del self._agg[k]
        try:
            self.q.put_nowait(ev)
        except asyncio.QueueFull:
            self.dropped += 1

    async def _take(self):
        """Token bucket in front of the API writes (client rate limiter on the event client)."""
        while True:
            now = time.monotonic()
            self._tokens = min(self.burst, self._tokens + (now - self._last) * self.qps)
            self._last = now
            if self._tokens >= 1.0:
                self._tokens -= 1.0
                return
            await asyncio.sleep((1.0 - self._tokens) / self.qps)

    async def _work(self):
        while True:
            ev = await self.q.get()
            if self.qps > 0:
                await self._take()
            upd = ev.pop("_update", False)
            try:
                if upd:
                    await self.client.patch("events", ev["metadata"]["name"],
                                            {"count": ev["count"], "lastTimestamp": ev["lastTimestamp"]},
                                            ev["metadata"]["namespace"], decode=False)
                else:
                    await self.client.create("events", ev, ev["metadata"]["namespace"], decode=False)
                self.sent += 1
            except Exception as e:  # events are best effort
                log.debug("event write failed: %s", e)

    async def flush(self, timeout=5.0):
        t = time.monotonic() + timeout
        while not self.q.empty() and time.monotonic() < t:
            await asyncio.sleep(0.01)
