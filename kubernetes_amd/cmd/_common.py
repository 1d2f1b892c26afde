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
        # a signal during startup (informer syncs, leader election) ends the process too,
        # without waiting for the component to finish starting
        starting = asyncio.ensure_future(main_coro_factory())
        stopping = asyncio.ensure_future(stop.wait())
        await asyncio.wait({starting, stopping}, return_when=asyncio.FIRST_COMPLETED)
        if not starting.done():
            starting.cancel()
            try:
                await starting
            except BaseException:       # noqa: BLE001 - cancelled startup, exiting anyway
                pass
            return
        stopping.cancel()
        comp = starting.result()
        tune_gc()
        await stop.wait()
        closer = getattr(comp, "stop", None)
        if closer is not None:
            await closer()
        # cancel what is left and give it a bounded time: a task that swallows its cancellation
        # (asyncio.wait_for on 3.10 can) must not keep a SIGTERMed component alive
        rest = [t for t in asyncio.all_tasks() if t is not asyncio.current_task() and not t.done()]
        for t in rest:
            t.cancel()
        if rest:
            _done, pending = await asyncio.wait(rest, timeout=5.0)
            if pending:
                import logging
                import sys
                for t in pending:
                    logging.getLogger("shutdown").warning("task ignored cancellation at shutdown: %r", t)
                    t.print_stack(file=sys.stderr)
                sys.stderr.flush()
                os._exit(0)
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


def unsupported(group, flag, default, type=str, why=""):
    """A reference flag whose subsystem this component does not have: the default still parses
    (reference command lines keep working), any other value is refused by `check_unsupported`
    instead of being silently ignored."""
    a = group.add_argument(flag, type=type, default=default,
                           help=f"unsupported: only the default ({default!r}) is accepted — {why}")
    a.kamd_unsupported = why
    return a


def check_unsupported(parser, args):
    """parser.error() for the first `unsupported` flag set to a non-default value."""
    for a in parser._actions:
        why = getattr(a, "kamd_unsupported", None)
        if why is None:
            continue
        v = getattr(args, a.dest, a.default)
        default = a.type(a.default) if isinstance(a.default, str) and a.type not in (None, str) else a.default
        if v != default:
            parser.error(f"{a.option_strings[0]}={v!r} is not supported here: {why}")


def deprecated_noop(group, flag, default, type=str, ref=""):
    """A flag the reference itself marks deprecated and ignores (its `MarkDeprecated(...,
    "...no-op...")`): accepted with any value, as there."""
    return group.add_argument(flag, type=type, default=default,
                              help=f"deprecated; a no-op in the reference too ({ref})")
