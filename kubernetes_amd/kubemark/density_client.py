"""Request-issuing helper processes for the density load generator.

The density runner (kubemark/density.py) observes pods on ONE watch and, in the reference's
e2e test, issues its creates and deletes from many goroutines. In one Python process the
issuing side competes with the watch for the event loop: 64 creates and 64 deletes per step are
~10 ms of client CPU in the rank. With `client_procs=K` the rank hands each step's creates and
deletes to K helper processes (this module) that issue them over their own HTTP connections,
while the rank's loop only watches. The create timestamp of each pod is taken in the helper
just before its request is sent, on CLOCK_MONOTONIC, which is system-wide on Linux, so startup
latency (create sent -> Running observed) keeps its definition.

Protocol: one JSON line per request on a unix socket, one JSON line per reply.
  {"op": "create", "ns", "names", "labels", "gpus", "annotations"} -> {"sent": {name: t}, "lat": [s]}
  {"op": "delete", "ns", "names"}                                  -> {"lat": [s]}
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import time


async def _serve(master, path, concurrency):
    from ..client.rest import APIStatusError, Client
    from .density import gpu_pod
    client = Client(master, max_conns=concurrency)
    sem = asyncio.Semaphore(concurrency)

    async def create(req, n, sent, lat):
        async with sem:
            sent[n] = t = time.monotonic()
            await client.create("pods", gpu_pod(n, req["ns"], req["labels"], req["gpus"],
                                                annotations=req.get("annotations")), req["ns"])
            lat.append(time.monotonic() - t)

    async def delete(req, n, lat):
        async with sem:
            t = time.monotonic()
            try:
                await client.delete("pods", n, req["ns"])
            except APIStatusError as e:
                if e.code != 404:
                    raise
            lat.append(time.monotonic() - t)

    async def handle(reader, writer):
        while True:
            line = await reader.readline()
            if not line:
                break
            req = json.loads(line)
            sent, lat = {}, []
            try:
                if req["op"] == "create":
                    await asyncio.gather(*(create(req, n, sent, lat) for n in req["names"]))
                    out = {"sent": sent, "lat": lat}
                else:
                    await asyncio.gather(*(delete(req, n, lat) for n in req["names"]))
                    out = {"lat": lat}
            except Exception as e:  # noqa: BLE001 - reported to the runner, which fails the step
                out = {"error": repr(e)}
            writer.write(json.dumps(out).encode() + b"\n")
            await writer.drain()
        writer.close()

    srv = await asyncio.start_unix_server(handle, path)
    open(path + ".ready", "w").close()
    async with srv:
        await srv.serve_forever()


class HelperPool:
    """K helper processes and one connection to each (used by DensityRunner)."""

    def __init__(self, master, k, workdir, concurrency=64):
        import subprocess
        import sys
        self.paths = [os.path.join(workdir, f"density-client-{os.getpid()}-{i}.sock") for i in range(k)]
        env = dict(os.environ)
        env.pop("HIP_VISIBLE_DEVICES", None)
        self.procs = [subprocess.Popen([sys.executable, "-m", "kubernetes_amd.kubemark.density_client",
                                        "--master", master, "--socket", p, "--concurrency", str(concurrency)],
                                       env=env) for p in self.paths]
        self.conns = []

    async def start(self, timeout=60):
        end = time.monotonic() + timeout
        for p, proc in zip(self.paths, self.procs):
            while not os.path.exists(p + ".ready"):
                if proc.poll() is not None or time.monotonic() > end:
                    raise RuntimeError(f"density client {p} did not start (exit {proc.poll()})")
                await asyncio.sleep(0.02)
            self.conns.append(await asyncio.open_unix_connection(p))
        return self

    async def call(self, op, ns, names, **kw):
        """Split `names` over the helpers; returns (merged sent-times, latencies)."""
        k = len(self.conns)
        parts = [names[i::k] for i in range(k)]
        for (_, w), part in zip(self.conns, parts):
            w.write(json.dumps(dict(kw, op=op, ns=ns, names=part)).encode() + b"\n")
        sent, lat = {}, []
        for (r, _), part in zip(self.conns, parts):
            out = json.loads(await r.readline())
            if "error" in out:
                raise RuntimeError(f"density client {op} failed: {out['error']}")
            sent.update(out.get("sent") or {})
            lat += out.get("lat") or []
        return sent, lat

    async def stop(self):
        for _, w in self.conns:
            w.close()
        for p in self.procs:
            p.terminate()
        for p in self.procs:
            try:
                p.wait(10)
            except Exception:  # noqa: BLE001
                p.kill()
        for path in self.paths:
            for f in (path, path + ".ready"):
                try:
                    os.unlink(f)
                except OSError:
                    pass


def main(argv=None):
    ap = argparse.ArgumentParser("density-client")
    ap.add_argument("--master", required=True)
    ap.add_argument("--socket", required=True)
    ap.add_argument("--concurrency", type=int, default=64)
    a = ap.parse_args(argv)
    from ..cmd._common import tune_gc
    tune_gc()
    asyncio.run(_serve(a.master, a.socket, a.concurrency))


if __name__ == "__main__":
    main()
