"""Same write-path workload against an API server running in its own process(es)
(`python -m kubernetes_amd.cmd.apiserver [--workers N]`), driven by several client processes,
so the numbers are server-side only.

    python benchmarks/apiserver_remote.py --pods 8000 --client-procs 4 --extra "--workers 4"
"""
import argparse
import asyncio
import multiprocessing as mp
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from kubernetes_amd.client.rest import Client  # noqa: E402


async def run(url, a, proc, start_at):
    ws = []
    for _ in range(a.watchers):
        w = await Client(url).watch("pods", None, "0")

        async def drain(w=w):
            async for _ in w:
                pass
        ws.append(asyncio.ensure_future(drain()))
    clients = [Client(url) for _ in range(a.clients)]
    n_per = a.pods // a.client_procs // a.clients

    async def worker(ci, c):
        for i in range(n_per):
            name = f"p{proc}-{ci}-{i}"
            if a.events_only:
                # the kubelet/scheduler event mix: 5 events per pod (Scheduled, Pulled, Created,
                # Started, Killing), each a POST of a new Event
                for reason in ("Scheduled", "Pulled", "Created", "Started", "Killing"):
                    await c.create("events", {
                        "metadata": {"name": f"{name}.{reason.lower()}", "namespace": "default"},
                        "involvedObject": {"kind": "Pod", "namespace": "default", "name": name,
                                           "uid": "u-" + name, "apiVersion": "v1", "resourceVersion": "1"},
                        "reason": reason, "message": f"{reason} pod {name}", "type": "Normal",
                        "source": {"component": "kubelet", "host": "n0"}, "count": 1,
                        "firstTimestamp": "2026-01-01T00:00:00Z", "lastTimestamp": "2026-01-01T00:00:00Z"})
                continue
            p = await c.create("pods", {"metadata": {"name": name, "namespace": "default"},
                                        "spec": {"containers": [{"name": "c", "image": "x",
                                                                 "resources": {"limits": {"amd.com/gpu": "1"}}}]}})
            er = p["spec"]["extendedResources"][0]["name"]
            await c.bind("default", name, "n0", {er: {"resources": [f"g-{proc}-{ci}-{i}"]}})
            await c.patch("pods", name, {"status": {"phase": "Running"}}, "default", "merge", "status")
            await c.delete("pods", name, "default")
            await c.delete("pods", name, "default", grace_period=0)
    while time.time() < start_at:
        await asyncio.sleep(0.005)
    t = time.perf_counter()
    await asyncio.gather(*(worker(i, c) for i, c in enumerate(clients)))
    return time.perf_counter() - t, n_per * a.clients


def _proc(args):
    url, a, proc, start_at = args
    return asyncio.run(run(url, a, proc, start_at))


async def _setup(url):
    c = Client(url)
    await c.create("nodes", {"metadata": {"name": "n0"}})
    await c.close()


def _server_cpu(pid):
    """User+system CPU seconds of the API server and every process under it (workers, store)."""
    import psutil
    root = psutil.Process(pid)
    tot = 0.0
    for q in [root] + root.children(recursive=True):
        try:
            t = q.cpu_times()
            tot += t.user + t.system
        except psutil.NoSuchProcess:
            pass
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pods", type=int, default=4000)
    ap.add_argument("--clients", type=int, default=64, help="concurrent clients per client process")
    ap.add_argument("--client-procs", type=int, default=1)
    ap.add_argument("--watchers", type=int, default=3)
    ap.add_argument("--extra", default="")
    ap.add_argument("--events-only", action="store_true", help="5 Event creates per pod instead of the pod lifecycle")
    a = ap.parse_args()
    d = tempfile.mkdtemp()
    pf = os.path.join(d, "port")
    env = dict(os.environ, PYTHONPATH=ROOT)
    p = subprocess.Popen([sys.executable, "-m", "kubernetes_amd.cmd.apiserver", "--port", "0", "--port-file", pf] + a.extra.split(),
                         env=env)
    while not os.path.exists(pf):
        time.sleep(0.05)
    try:
        url = f"http://127.0.0.1:{open(pf).read()}"
        asyncio.run(_setup(url))
        start_at = time.time() + 1.0 + 0.2 * a.client_procs
        cpu0 = _server_cpu(p.pid)
        with mp.get_context("spawn").Pool(a.client_procs) as pool:
            res = pool.map(_proc, [(url, a, i, start_at) for i in range(a.client_procs)])
        cpu = _server_cpu(p.pid) - cpu0
        dt = max(r[0] for r in res)
        pods = sum(r[1] for r in res)
        print(f"{a.extra or 'single process'}: {pods / dt:.0f} pod-cycles/s, {pods * 5 / dt:.0f} writes/s, "
              f"{dt * 1e6 / (pods * 5):.1f} us/write, server CPU {cpu * 1e3 / pods:.3f} ms per pod-cycle "
              f"(all API server processes, store included)")
    finally:
        p.terminate()
        p.wait()


if __name__ == "__main__":
    main()
