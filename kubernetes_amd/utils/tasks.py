"""Fire-and-forget tasks that cannot be garbage-collected mid-flight.

asyncio keeps only weak references to tasks; a task whose awaited futures are reachable only
from itself (e.g. an in-flight HTTP request: StreamReaderProtocol holds its reader weakly) can
be collected as a reference cycle while still pending. `spawn` keeps a strong reference until
the task is done.
"""
from __future__ import annotations

import asyncio

_live: set = set()


def spawn(coro) -> asyncio.Task:
    t = asyncio.ensure_future(coro)
    _live.add(t)
    t.add_done_callback(_live.discard)
    return t
