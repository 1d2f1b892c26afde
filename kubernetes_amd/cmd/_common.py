"""Shared bits for the component entry points."""
from __future__ import annotations

import asyncio
import logging
import os
import signal


def setup_logging(v: int = 0):
    lvl = logging.WARNING if v <= 0 else (logging.INFO if v == 1 else logging.DEBUG)
    logging.basicConfig(level=lvl, format="%(asctime)s %(levelname).1s %(name)s] %(message)s")


def write_port_file(path, port):
    if path:
        tmp = path + ".tmp"
        with open(tmp, "w") as f:
            f.write(str(port))
        os.replace(tmp, path)


def tune_gc():
    """Long-running components allocate mostly acyclic JSON dicts (freed by refcounting), so the
    cyclic collector only adds pauses: a full collection over a large heap stalls the event loop
    for tens of ms (visible as API call p99 spikes). Young collections run 70x less often, and
    everything alive once the component is up moves to the permanent generation (`gc.freeze`).
    KAMD_GC_THRESHOLD="a,b,c" overrides the thresholds ("0" disables the collector)."""
    import gc
    v = os.environ.get("KAMD_GC_THRESHOLD", "50000,20,100")
    if v.strip() == "0":
        gc.disable()
    else:
        try:
            gc.set_threshold(*(int(x) for x in v.split(",")))
        except (TypeError, ValueError):
            pass
    gc.freeze()


def run_until_signal(main_coro_factory):
    """Run an asyncio component until SIGINT/SIGTERM."""
    async def runner():
        loop = asyncio.get_running_loop()
        stop = asyncio.Event()
        for s in (signal.SIGINT, signal.SIGTERM):
            try:
                loop.add_signal_handler(s, stop.set)
            except NotImplementedError:
                pass
        comp = await main_coro_factory()
        tune_gc()
        await stop.wait()
        closer = getattr(comp, "stop", None)
        if closer is not None:
            await closer()
    prof_dir = os.environ.get("KAMD_PROFILE_DIR")
    if prof_dir:
        # pprof-equivalent: whole-process cProfile dump at shutdown (reference: /debug/pprof)
        import cProfile
        import sys
        pr = cProfile.Profile()
        pr.enable()
        try:
            asyncio.run(runner())
        finally:
            pr.disable()
            os.makedirs(prof_dir, exist_ok=True)
            pr.dump_stats(os.path.join(prof_dir, os.path.basename(sys.argv[0]).replace(".py", "") + f".{os.getpid()}.prof"))
        return
    asyncio.run(runner())
