"""GPU payload service for hollow nodes running in their own processes.

kubemark runs every hollow node as a separate process (`cmd/kubemark/hollow-node.go`). The
density bench does the same, but only ONE process per MI355X should hold a HIP context (the
rank), so hollow-node processes do not run the GPU payload themselves: their stub runtime asks the
rank's `PayloadServer` over a unix socket, which launches the HIP vector_add on the rank's GPU and
answers pass/fail. One byte each way per container start; requests on a connection are answered
in order, so a client keeps one connection and a FIFO of pending futures.
"""
from __future__ import annotations

import asyncio
import collections
import os


class PayloadServer:
    def __init__(self, run, path):
        self.run = run                  # () -> bool, e.g. ops.hip_kernels.Payload(dev).run
        self.path = path
        self.runs = 0
        self.failures = 0
        self._srv = None

    async def _serve(self, reader, writer):
        try:
            while True:
                req = await reader.read(4096)
                if not req:
                    break
                out = bytearray()
                for _ in range(len(req)):            # one byte per request
                    ok = False
                    self.runs += 1
                    try:
                        ok = bool(self.run())
                    except Exception:  # noqa: BLE001 - a crashing payload is a failed container
                        ok = False
                    if not ok:
                        self.failures += 1
                    out += b"1" if ok else b"0"
                writer.write(bytes(out))
        except (ConnectionError, asyncio.CancelledError):
            pass
        finally:
            writer.close()

    async def start(self):
        if os.path.exists(self.path):
            os.unlink(self.path)
        self._srv = await asyncio.start_unix_server(self._serve, self.path)
        return self

    async def stop(self):
        if self._srv is not None:
            self._srv.close()
            await self._srv.wait_closed()
        try:
            os.unlink(self.path)
        except OSError:
            pass


class PayloadClient:
    """Async callable for `StubRuntime(payload=...)`: `await client(opts)` -> bool."""

    def __init__(self, path):
        self.path = path
        self._w = None
        self._pending: collections.deque = collections.deque()
        self._reader_task = None
        self._lock = asyncio.Lock()

    async def _connect(self):
        r, w = await asyncio.open_unix_connection(self.path)
        self._w = w
        self._reader_task = asyncio.ensure_future(self._read(r))

    async def _read(self, r):
        try:
            while True:
                data = await r.read(4096)
                if not data:
                    break
                for b in data:
                    fut = self._pending.popleft()
                    if not fut.done():
                        fut.set_result(b == ord("1"))
        finally:
            while self._pending:
                f = self._pending.popleft()
                if not f.done():
                    f.set_exception(ConnectionError("payload server went away"))
            self._w = None

    async def __call__(self, opts=None) -> bool:
        if self._w is None:
            async with self._lock:
                if self._w is None:
                    await self._connect()
        fut = asyncio.get_running_loop().create_future()
        self._pending.append(fut)
        self._w.write(b"R")
        return await fut

    async def close(self):
        if self._w is not None:
            self._w.close()
        if self._reader_task is not None:
            self._reader_task.cancel()
