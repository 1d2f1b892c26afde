"""/debug/pprof equivalents for the Python components.

Parity: `staging/src/k8s.io/apiserver/pkg/server/routes/profiling.go:30-36` (apiserver),
`plugin/cmd/kube-scheduler/app/server.go:469-512`, `pkg/kubelet/server/server.go:295-402`:
  * /debug/pprof/               index
  * /debug/pprof/profile?seconds=N   CPU profile of the event loop thread for N s (cProfile,
                                     pstats text sorted by cumulative time; `?sort=tottime`)
  * /debug/pprof/goroutine      every asyncio task's stack + every thread's stack
  * /debug/pprof/heap           tracemalloc top allocations (starts tracing on first call)
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


async def handle_debug(req):
    """Returns a Response for /debug/pprof/* paths, else None."""
    p = req.path
    if not p.startswith("/debug/pprof"):
        return None
    sub = p[len("/debug/pprof"):].strip("/")
    if sub == "":
        return Response(200, b"/debug/pprof/profile?seconds=N\n/debug/pprof/goroutine\n/debug/pprof/heap\n", "text/plain")
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
