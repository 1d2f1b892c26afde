"""Work queues and the parallelizer.

Parity: `staging/src/k8s.io/client-go/util/workqueue/{queue.go,delaying_queue.go,rate_limitting_queue.go,
default_rate_limiters.go,parallelizer.go:29}`.

Semantics kept from the reference: an item is never processed by two workers at once
(dirty/processing sets); re-adding an item while it is processing re-queues it after
`done()`; per-item exponential backoff (5 ms .. 1000 s) combined with an overall token bucket.
"""
from __future__ import annotations

import asyncio
import heapq
import itertools
import time
from concurrent.futures import ThreadPoolExecutor


class WorkQueue:
    def __init__(self, name=""):
        self.name = name
        self._queue: list = []
        self._dirty: set = set()
        self._processing: set = set()
        self._cond = asyncio.Condition()
        self._shutting_down = False
        self._waiters = 0
        self._ev = asyncio.Event()
        self.adds = 0

    def add(self, item):
        if self._shutting_down or item in self._dirty:
            return
        self.adds += 1
        self._dirty.add(item)
        if item in self._processing:
            return
        self._queue.append(item)
        self._ev.set()

    def __len__(self):
        return len(self._queue)

    async def get(self):
        """Returns (item, shutdown)."""
        while not self._queue:
            if self._shutting_down:
                return None, True
            self._ev.clear()
            await self._ev.wait()
        item = self._queue.pop(0)
        self._processing.add(item)
        self._dirty.discard(item)
        return item, False

    def get_nowait(self):
        if not self._queue:
            return None
        item = self._queue.pop(0)
        self._processing.add(item)
        self._dirty.discard(item)
        return item

    def done(self, item):
        self._processing.discard(item)
        if item in self._dirty:
            self._queue.append(item)
            self._ev.set()

    def shutdown(self):
        self._shutting_down = True
        self._ev.set()

    @property
    def shutting_down(self):
        return self._shutting_down


class ItemExponentialFailureRateLimiter:
    def __init__(self, base=0.005, cap=1000.0):
        self.base, self.cap = base, cap
        self.failures = {}

    def when(self, item):
        n = self.failures.get(item, 0)
        self.failures[item] = n + 1
        return min(self.base * (2 ** n), self.cap)

    def forget(self, item):
        self.failures.pop(item, None)

    def num_requeues(self, item):
        return self.failures.get(item, 0)


class BucketRateLimiter:
    def __init__(self, qps=10.0, burst=100):
        self.qps, self.burst = qps, burst
        self.tokens = float(burst)
        self.t = time.monotonic()
        self.reserved_until = 0.0

    def when(self, item):
        now = time.monotonic()
        self.tokens = min(self.burst, self.tokens + (now - self.t) * self.qps)
        self.t = now
        if self.tokens >= 1:
            self.tokens -= 1
            return 0.0
        self.tokens -= 1
        return -self.tokens / self.qps

    def forget(self, item):
        pass

    def num_requeues(self, item):
        return 0


class MaxOfRateLimiter:
    def __init__(self, *limiters):
        self.limiters = limiters

    def when(self, item):
        return max(l.when(item) for l in self.limiters)

    def forget(self, item):
        for l in self.limiters:
            l.forget(item)

    def num_requeues(self, item):
        return max(l.num_requeues(item) for l in self.limiters)


def default_controller_rate_limiter():
    return MaxOfRateLimiter(ItemExponentialFailureRateLimiter(0.005, 1000.0), BucketRateLimiter(10, 100))


class RateLimitingQueue(WorkQueue):
    """Delaying + rate limiting queue."""

    def __init__(self, name="", rate_limiter=None):
        super().__init__(name)
        self.rl = rate_limiter or default_controller_rate_limiter()
        self._heap = []
        self._seq = itertools.count()
        self._timer = None

    def add_after(self, item, delay):
        if delay <= 0:
            self.add(item)
            return
        heapq.heappush(self._heap, (time.monotonic() + delay, next(self._seq), item))
        self._arm()

    def _arm(self):
        if not self._heap:
            return
        loop = asyncio.get_event_loop()
        when = self._heap[0][0]
        if self._timer is not None:
            if self._timer.when() <= loop.time() + (when - time.monotonic()) + 1e-4:
                return
            self._timer.cancel()
        self._timer = loop.call_later(max(0.0, when - time.monotonic()), self._fire)

    def _fire(self):
        self._timer = None
        now = time.monotonic()
        while self._heap and self._heap[0][0] <= now:
            _, _, item = heapq.heappop(self._heap)
            self.add(item)
        self._arm()

    def add_rate_limited(self, item):
        self.add_after(item, self.rl.when(item))

    def forget(self, item):
        self.rl.forget(item)

    def num_requeues(self, item):
        return self.rl.num_requeues(item)

    def shutdown(self):
        super().shutdown()
        if self._timer:
            self._timer.cancel()


_POOL = None


def parallelize(workers: int, pieces: int, fn):
    """`workqueue.Parallelize(workers, pieces, doWorkPiece)` for CPU-side fan-out.

    With the GIL, thread fan-out only pays when `fn` releases it (native code); the
    scheduler's hot path therefore calls this only above a size threshold and otherwise
    runs serially (on one node parallel-over-nodes gains nothing)."""
    global _POOL
    if pieces <= 0:
        return
    if workers <= 1 or pieces < 64:
        for i in range(pieces):
            fn(i)
        return
    if _POOL is None:
        _POOL = ThreadPoolExecutor(max_workers=16, thread_name_prefix="parallelize")
    list(_POOL.map(fn, range(pieces)))
