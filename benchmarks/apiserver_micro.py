"""API server write-path microbenchmark: create → bind → status patch → delete per pod,
from C concurrent clients, with W watchers attached (scheduler/kubelet/density roles)."""
import argparse
import asyncio
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kubernetes_amd.apiserver.server import APIServer  # noqa: E402
from kubernetes_amd.client.rest import Client  # noqa: E402


async def main(a):
    s = APIServer()
    port = await s.start()
    url = f"http://127.0.0.1:{port}"
    c0 = Client(url)
    await c0.create("nodes", {"metadata": {"name": "n0"}})
    watchers = []
    for i in range(a.watchers):
        w = await Client(url).watch("pods", None, "0")
        watchers.append(asyncio.ensure_future(_drain(w)))
    clients = [Client(url) for _ in range(a.clients)]
    n_per = a.pods // a.clients

    async def worker(ci, c):
        for i in range(n_per):
            name = f"p{ci}-{i}"
            p = await c.create("pods", {"metadata": {"name": name, "namespace": "default"},
                                        "spec": {"containers": [{"name": "c", "image": "x",
                                                                 "resources": {"limits": {"amd.com/gpu": "1"}}}]}})
            er = p["spec"]["extendedResources"][0]["name"]
            await c.bind("default", name, "n0", {er: {"resources": [f"g-{ci}-{i}"]}})
            await c.patch("pods", name, {"status": {"phase": "Running"}}, "default", "merge", "status")
            await c.delete("pods", name, "default")
            await c.delete("pods", name, "default", grace_period=0)
    pr = cProfile.Profile() if a.profile else None
    t = time.perf_counter()
    if pr:
        pr.enable()
    await asyncio.gather(*(worker(i, c) for i, c in enumerate(clients)))
    if pr:
        pr.disable()
    dt = time.perf_counter() - t
    writes = a.pods * 5
    print(f"pods={a.pods} clients={a.clients} watchers={a.watchers}: {a.pods / dt:.0f} pod-cycles/s, "
          f"{writes / dt:.0f} writes/s, {dt * 1e6 / writes:.1f} us/write")
    if pr:
        pstats.Stats(pr).sort_stats("tottime").print_stats(25)
    for w in watchers:
        w.cancel()
    await s.stop()


async def _drain(w):
    async for _ in w:
        pass


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--pods", type=int, default=4000)
    ap.add_argument("--clients", type=int, default=32)
    ap.add_argument("--watchers", type=int, default=3)
    ap.add_argument("--profile", action="store_true")
    asyncio.run(main(ap.parse_args()))
