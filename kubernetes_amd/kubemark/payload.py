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
    """`run` is `() -> bool` (one start) or an object with `run_batch(k) -> [bool]` (e.g.
    `ops.hip_kernels.Payload`): the starts that arrived in one read are run as ONE batch —
    k kernel launches, one verify kernel, one stream sync — on a worker thread, so the rank's
    event loop keeps serving its watches while the GPU works."""

    def __init__(self, run, path):
        self.run = run
        self._batch = getattr(run, "run_batch", None) or getattr(getattr(run, "__self__", None), "run_batch", None)
        self.path = path
        self.runs = 0
        self.failures = 0
        self.batches = 0
        self._srv = None
        from concurrent.futures import ThreadPoolExecutor
        self._pool = ThreadPoolExecutor(1, thread_name_prefix="payload")   # one HIP caller at a time

    def _run_many(self, k):
        if self._batch is not None:
            return self._batch(k)
        out = []
        for _ in range(k):
            try:
                out.append(bool(self.run()))
            except Exception:  # noqa: BLE001 - a crashing payload is a failed container
                out.append(False)
        return out

    async def _serve(self, reader, writer):
        loop = asyncio.get_running_loop()
        try:
            while True:
                req = await reader.read(4096)
                if not req:
                    break
                k = len(req)                         # one byte per request
                try:
                    oks = await loop.run_in_executor(self._pool, self._run_many, k)
                except Exception:  # noqa: BLE001
                    oks = [False] * k
                self.runs += k
                self.batches += 1
                self.failures += sum(1 for ok in oks if not ok)
                writer.write(b"".join(b"1" if ok else b"0" for ok in oks))
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
        self._pool.shutdown(wait=True)
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
        self._queued = 0

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
        loop = asyncio.get_running_loop()
        fut = loop.create_future()
        self._pending.append(fut)
        # container starts issued in one loop iteration leave in ONE write -> one GPU batch
        if not self._queued:
            loop.call_soon(self._flush)
        self._queued += 1
        return await fut

    def _flush(self):
        n, self._queued = self._queued, 0
        if n and self._w is not None:
            self._w.write(b"R" * n)

    async def close(self):
        if self._w is not None:
            self._w.close()
        if self._reader_task is not None:
            self._reader_task.cancel()
