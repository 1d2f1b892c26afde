"""Same write-path workload against an API server running in its own process
(`python -m kubernetes_amd.cmd.apiserver`), so the numbers are server-side only."""
import argparse
import asyncio
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from kubernetes_amd.client.rest import Client  # noqa: E402


async def run(url, a):
    c0 = Client(url)
    await c0.create("nodes", {"metadata": {"name": "n0"}})
    ws = []
    for _ in range(a.watchers):
        w = await Client(url).watch("pods", None, "0")

        async def drain(w=w):
            async for _ in w:
                pass
        ws.append(asyncio.ensure_future(drain()))
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
    t = time.perf_counter()
    await asyncio.gather(*(worker(i, c) for i, c in enumerate(clients)))
    dt = time.perf_counter() - t
    print(f"{a.pods / dt:.0f} pod-cycles/s, {a.pods * 5 / dt:.0f} writes/s, {dt * 1e6 / (a.pods * 5):.1f} us/write")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pods", type=int, default=4000)
    ap.add_argument("--clients", type=int, default=64)
    ap.add_argument("--watchers", type=int, default=3)
    ap.add_argument("--extra", default="")
    a = ap.parse_args()
    d = tempfile.mkdtemp()
    pf = os.path.join(d, "port")
    env = dict(os.environ, PYTHONPATH=ROOT)
    p = subprocess.Popen([sys.executable, "-m", "kubernetes_amd.cmd.apiserver", "--port", "0", "--port-file", pf] + a.extra.split(),
                         env=env)
    while not os.path.exists(pf):
        time.sleep(0.05)
    try:
        asyncio.run(run(f"http://127.0.0.1:{open(pf).read()}", a))
    finally:
        p.terminate()
        p.wait()


if __name__ == "__main__":
    main()
