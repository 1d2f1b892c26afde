"""/debug/pprof equivalents for the Python components.

Parity: `staging/src/k8s.io/apiserver/pkg/server/routes/profiling.go:30-36` (apiserver),
`plugin/cmd/kube-scheduler/app/server.go:469-512`, `pkg/kubelet/server/server.go:295-402`:
  * /debug/pprof/               index
  * /debug/pprof/profile?seconds=N   CPU profile of the event loop thread for N s (cProfile,
                                     pstats text sorted by cumulative time; `?sort=tottime`)
  * /debug/pprof/goroutine      every asyncio task's stack + every thread's stack
  * /debug/pprof/heap           tracemalloc top allocations (starts tracing on first call)
  * /debug/pprof/block          with --contention-profiling: where the event loop was blocked
                                (Go's block/mutex profile; here the one thing every request
                                contends for is the loop thread, so the profile samples its stack
                                whenever it has not come back to the loop for > 20 ms)
"""
from __future__ import annotations

import asyncio
import cProfile
import io
import pstats
import sys
import threading
import traceback

from .httpserver import Response

_busy = asyncio.Lock() if sys.version_info >= (3, 10) else None
_block = None


class BlockProfiler:
    """A watchdog thread plus a heartbeat callback on the loop: when the heartbeat is late by
    more than `threshold` s, the loop thread's current stack is sampled; samples are aggregated
    per stack with the blocked time they account for."""

    def __init__(self, loop, threshold=0.02, interval=0.005):
        import time
        self.loop, self.threshold, self.interval = loop, threshold, interval
        self.beat = time.monotonic()
        self.samples: dict = {}           # stack text -> [samples, blocked seconds]
        self.loop_thread = None
        self._stop = threading.Event()

    def _heartbeat(self):
        import time
        self.beat = time.monotonic()
        if not self._stop.is_set():
            self.loop.call_later(self.interval, self._heartbeat)

    def _watch(self):
        import time
        while not self._stop.wait(self.interval):
            late = time.monotonic() - self.beat - self.interval
            if late < self.threshold:
                continue
            fr = sys._current_frames().get(self.loop_thread)
            if fr is None:
                continue
            key = "".join(traceback.format_stack(fr, limit=12))
            e = self.samples.setdefault(key, [0, 0.0])
            e[0] += 1
            e[1] += self.interval

    def start(self):
        self.loop_thread = threading.get_ident()     # called on the loop thread
        self.loop.call_soon(self._heartbeat)
        threading.Thread(target=self._watch, name="block-profiler", daemon=True).start()
        return self

    def stop(self):
        self._stop.set()

    def report(self, limit=20):
        top = sorted(self.samples.items(), key=lambda kv: -kv[1][1])[:limit]
        total = sum(v[1] for v in self.samples.values())
        out = [f"event loop blocked > {self.threshold * 1e3:.0f} ms: {total * 1e3:.0f} ms sampled "
               f"over {sum(v[0] for v in self.samples.values())} samples\n"]
        for stack, (n, secs) in top:
            out.append(f"--- {secs * 1e3:.0f} ms ({n} samples)\n{stack}")
        return "\n".join(out)


def enable_contention_profiling(loop=None):
    """--contention-profiling: start the block profiler on the running loop (idempotent)."""
    global _block
    if _block is None:
        _block = BlockProfiler(loop or asyncio.get_running_loop()).start()
    return _block


async def handle_debug(req):
    """Returns a Response for /debug/pprof/* paths, else None."""
    p = req.path
    if not p.startswith("/debug/pprof"):
        return None
    sub = p[len("/debug/pprof"):].strip("/")
    if sub == "":
        return Response(200, b"/debug/pprof/profile?seconds=N\n/debug/pprof/goroutine\n/debug/pprof/heap\n"
                             b"/debug/pprof/block\n", "text/plain")
    if sub == "block":
        if _block is None:
            return Response(404, b"contention profiling is off (--contention-profiling)\n", "text/plain")
        return Response(200, _block.report(int(req.query.get("limit") or 20)).encode(), "text/plain")
    if sub == "profile":
        secs = min(float(req.query.get("seconds") or 10), 120.0)
        sort = req.query.get("sort") or "cumulative"
        if _busy.locked():
            return Response(409, b"a profile is already being collected\n", "text/plain")
        async with _busy:
            pr = cProfile.Profile()
            pr.enable()
            try:
                await asyncio.sleep(secs)
            finally:
                pr.disable()
        out = io.StringIO()
        pstats.Stats(pr, stream=out).sort_stats(sort).print_stats(int(req.query.get("limit") or 60))
        return Response(200, out.getvalue().encode(), "text/plain")
    if sub == "goroutine":
        out = io.StringIO()
        for t in asyncio.all_tasks():
            out.write(f"task {t.get_name()} {t!r}\n")
            for fr in t.get_stack(limit=20):
                out.write("".join(traceback.format_stack(fr, limit=1)))
            out.write("\n")
        frames = sys._current_frames()
        for th in threading.enumerate():
            fr = frames.get(th.ident)
            out.write(f"thread {th.name} (daemon={th.daemon})\n")
            if fr is not None:
                out.write("".join(traceback.format_stack(fr)))
            out.write("\n")
        return Response(200, out.getvalue().encode(), "text/plain")
    if sub == "heap":
        import tracemalloc
        if not tracemalloc.is_tracing():
            tracemalloc.start(10)
            return Response(200, b"tracemalloc started; request again for a snapshot\n", "text/plain")
        snap = tracemalloc.take_snapshot()
        lines = [str(s) for s in snap.statistics("lineno")[: int(req.query.get("limit") or 40)]]
        return Response(200, ("\n".join(lines) + "\n").encode(), "text/plain")
    return Response(404, b"unknown profile\n", "text/plain")
