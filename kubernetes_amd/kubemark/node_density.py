"""Single-node density and kubelet resource usage (the reference's `test/e2e_node/density_test.go`
and `resource_usage_test.go`, BASELINE.md "node perf" rows).

One real kubelet runs in its own process (process runtime: every container is a real child
process) against an API server + scheduler in other processes, and a sampler reads the kubelet
process's CPU and RSS (the reference samples kubelet and runtime with a standalone cAdvisor).
Two workloads, as in the reference:
  * batch: N pods created at once; per-pod create → Running latency percentiles and the time
    until the whole batch runs (thresholds p50/p90/p99 ≤ 16/18/20 s, batch ≤ 25 s for N=10,
    `density_test.go:71-91`);
  * sequential: with B background pods running, N pods created one after the other, each
    waited for (thresholds 5/9/10 s, `density_test.go:213-228`);
  * the kubelet's CPU (cores) p50/p95 and RSS over the density run (thresholds 0.30/0.50 cores
    and 100 MiB, `density_test.go:76-83`), sampled every second like the reference's standalone
    cAdvisor (`resource_collector.go:56`, housekeeping 1 s);
  * steady-state resource tracking with every pod running (`resource_usage_test.go:65-78,
    136-182`: settle, then monitor; kubelet limits for 10 pods p50 ≤ 0.30 / p95 ≤ 0.35 cores,
    RSS ≤ 200 MiB), plus kubelet CPU-seconds spent per started pod;
  * `--runtime remote`: the kubelet talks CRI to a separate `kamd-cri` process (the reference's
    dockershim/docker split), whose CPU and RSS are tracked too (thresholds p50 ≤ 0.40 / p95 ≤
    0.60 cores, RSS ≤ 500 MiB, `density_test.go:76-83`);
  * `--gpu-pods N` (MI355X): the real `amd.com/gpu` device plugin runs as its own process on the
    node's GPUs (AMD SMI), and with the background pods running N pods requesting one GPU each
    run the HIP `vector_add` kernel (`kubernetes-amd/hip-vector-add`) through ResourceV2, the
    scheduler's device binding, the DeviceManager and kamd-runc's device injection — first one
    after the other (create → Running and create → Succeeded per pod, the sequential SLO applied
    to create → Running), then all N at once (each waits for the GPU the previous one frees:
    the makespan and per-pod completion percentiles).

    python -m kubernetes_amd.kubemark.node_density --batch 10 --sequential 10 --background 50
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import subprocess
import sys
import tempfile
import time

from ..client.rest import Client
from .density import pct

THRESHOLDS = {"batch": {"p50": 16.0, "p90": 18.0, "p99": 20.0, "all": 25.0},
              "sequential": {"p50": 5.0, "p90": 9.0, "p99": 10.0},
              "kubelet_cpu": {"p50": 0.30, "p95": 0.50}, "kubelet_rss_mib": 100.0,
              "steady_kubelet_cpu": {"p50": 0.30, "p95": 0.35}, "steady_kubelet_rss_mib": 200.0,
              "runtime_cpu": {"p50": 0.40, "p95": 0.60}, "runtime_rss_mib": 500.0}


def _spawn(args, tmp, name):
    env = dict(os.environ)
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    env["PYTHONPATH"] = root + os.pathsep + env.get("PYTHONPATH", "")
    return subprocess.Popen([sys.executable, "-m"] + args, env=env, stdout=subprocess.DEVNULL,
                            stderr=open(os.path.join(tmp, f"{name}.log"), "w"))


class Sampler:
    """CPU (cores) and RSS of one process, sampled every `period` seconds."""

    def __init__(self, pid, period=1.0):
        import psutil
        self.p = psutil.Process(pid)
        self.period = period
        self.cpu, self.rss = [], []
        self._task = None

    def cpu_seconds(self):
        return sum(self.p.cpu_times()[:2])

    def reset(self):
        self.cpu, self.rss = [], []

    async def _run(self):
        last_t, last_cpu = time.monotonic(), self.cpu_seconds()
        while True:
            await asyncio.sleep(self.period)
            t, cpu = time.monotonic(), self.cpu_seconds()
            self.cpu.append((cpu - last_cpu) / max(t - last_t, 1e-6))
            self.rss.append(self.p.memory_info().rss)
            last_t, last_cpu = t, cpu

    def start(self):
        self._task = asyncio.ensure_future(self._run())
        return self

    def stop(self):
        if self._task:
            self._task.cancel()


def _pod(name, sleep=3600):
    return {"metadata": {"name": name, "labels": {"density": "node"}},
            "spec": {"restartPolicy": "Never", "terminationGracePeriodSeconds": 1,
                     "containers": [{"name": "c", "image": "busybox", "command": ["sleep", str(sleep)]}]}}


def _gpu_pod(name):
    from ..api import core
    return {"metadata": {"name": name, "labels": {"density": "gpu"}},
            "spec": {"restartPolicy": "Never", "terminationGracePeriodSeconds": 1,
                     "containers": [{"name": "vector-add", "image": "kubernetes-amd/hip-vector-add",
                                     "resources": {"limits": {core.AMD_GPU: "1"}}}]}}


async def _wait_phases(client, ns, names, phases, timeout):
    """{name: {phase: first time observed}} for the given phases, until every name reached the
    last one (or failed) or `timeout`."""
    seen = {n: {} for n in names}
    last = phases[-1]
    lst = await client.list("pods", ns)
    now = time.monotonic()
    for p in lst["items"]:
        ph = (p.get("status") or {}).get("phase")
        if p["metadata"]["name"] in seen and ph in phases:
            seen[p["metadata"]["name"]].setdefault(ph, now)
    w = await client.watch("pods", ns, lst["metadata"]["resourceVersion"])
    end = time.monotonic() + timeout

    def done():
        return all(last in v or "Failed" in v for v in seen.values())

    async def drain():
        if done():
            return
        async for _, p in w:
            n = p["metadata"]["name"]
            ph = (p.get("status") or {}).get("phase")
            if n in seen and (ph in phases or ph == "Failed"):
                t = time.monotonic()
                seen[n].setdefault(ph, t)
                if ph in (last, "Failed"):
                    for q in phases:                # a phase the watch skipped counts as reached then
                        seen[n].setdefault(q, t)
            if done():
                return
    try:
        await asyncio.wait_for(drain(), max(0.1, end - time.monotonic()))
    except asyncio.TimeoutError:
        pass
    finally:
        w.close()
    return seen


async def _gpu_phase(c, ns, n, timeout):
    """Sequential then concurrent single-GPU HIP pods (see the module docstring)."""
    seq_run, seq_done, failed = [], [], []
    for i in range(n):
        name = f"gpu-seq-{i}"
        t0 = time.monotonic()
        await c.create("pods", _gpu_pod(name), ns)
        seen = (await _wait_phases(c, ns, [name], ("Running", "Succeeded"), timeout))[name]
        if "Failed" in seen or "Succeeded" not in seen:
            failed.append(name)
        else:
            seq_run.append(seen["Running"] - t0)
            seq_done.append(seen["Succeeded"] - t0)
        await c.delete("pods", name, ns, grace_period=0)
    names = [f"gpu-batch-{i}" for i in range(n)]
    t0 = time.monotonic()
    for name in names:
        await c.create("pods", _gpu_pod(name), ns)
    seen = await _wait_phases(c, ns, names, ("Running", "Succeeded"), timeout * max(1, n))
    done = [seen[x]["Succeeded"] - t0 for x in names if "Succeeded" in seen[x] and "Failed" not in seen[x]]
    failed += [x for x in names if "Succeeded" not in seen[x] or "Failed" in seen[x]]
    return {"pods": n, "failed": failed,
            "sequential": {"running_p50_s": round(pct(seq_run, .5), 3), "running_p90_s": round(pct(seq_run, .9), 3),
                           "running_p99_s": round(pct(seq_run, .99), 3),
                           "succeeded_p50_s": round(pct(seq_done, .5), 3),
                           "succeeded_p99_s": round(pct(seq_done, .99), 3)},
            "batch": {"makespan_s": round(max(done), 3) if len(done) == n else float("inf"),
                      "succeeded_p50_s": round(pct(done, .5), 3), "succeeded_p99_s": round(pct(done, .99), 3),
                      "gpu_pods_per_s": round(n / max(done), 2) if len(done) == n and max(done) > 0 else 0.0}}


async def _wait_running(client, ns, names, timeout):
    """name -> time observed Running (watch), within timeout."""
    seen = {}
    lst = await client.list("pods", ns)
    for p in lst["items"]:
        if (p.get("status") or {}).get("phase") == "Running":
            seen[p["metadata"]["name"]] = time.monotonic()
    w = await client.watch("pods", ns, lst["metadata"]["resourceVersion"])
    end = time.monotonic() + timeout

    async def drain():
        async for _, p in w:
            if (p.get("status") or {}).get("phase") == "Running":
                seen.setdefault(p["metadata"]["name"], time.monotonic())
            if all(n in seen for n in names):
                return
    try:
        await asyncio.wait_for(drain(), max(0.1, end - time.monotonic()))
    finally:
        w.close()
    return seen


async def _drain_pods(url):
    """Delete every pod and wait until the kubelet has confirmed each one gone (a graceful
    delete stays visible until its containers are stopped)."""
    c = Client(url)
    try:
        for p in (await c.list("pods"))["items"]:
            try:
                await c.delete("pods", p["metadata"]["name"], p["metadata"]["namespace"], grace_period=1)
            except Exception:      # noqa: BLE001 - already gone
                pass
        while (await c.list("pods"))["items"]:
            await asyncio.sleep(0.2)
    finally:
        await c.close()


async def run(batch=10, sequential=10, background=50, timeout=120.0, settle=2.0, monitor=10.0, period=1.0,
              runtime="process", gpu_pods=0):
    tmp = tempfile.mkdtemp(prefix="kamd-node-density-")
    pf = os.path.join(tmp, "api.port")
    procs = [_spawn(["kubernetes_amd.cmd.apiserver", "--port", "0", "--port-file", pf], tmp, "apiserver")]
    url = None
    try:
        t = time.time()
        while not os.path.exists(pf):
            if time.time() - t > 60:
                raise TimeoutError("apiserver did not start")
            await asyncio.sleep(0.05)
        url = f"http://127.0.0.1:{open(pf).read().strip()}"
        procs.append(_spawn(["kubernetes_amd.cmd.scheduler", "--master", url], tmp, "scheduler"))
        rt_args, rt_proc = ["--container-runtime", "process"], None
        if runtime == "remote":
            sock = os.path.join(tmp, "cri.sock")
            rt_proc = _spawn(["kubernetes_amd.cmd.cri", "--listen", sock, "--runtime", "process",
                              "--root-dir", os.path.join(tmp, "cri")], tmp, "cri")
            procs.append(rt_proc)
            t = time.time()
            while not os.path.exists(sock):
                if time.time() - t > 60:
                    raise TimeoutError("kamd-cri did not start")
                await asyncio.sleep(0.05)
            rt_args = ["--container-runtime", "remote", "--container-runtime-endpoint", f"unix://{sock}"]
        kl = _spawn(["kubernetes_amd.cmd.kubelet", "--api-servers", url, "--hostname-override", "density-node",
                     "--root-dir", os.path.join(tmp, "kubelet"), "--port", "0",
                     "--container-log-dir", "", "--max-pods", str(background + batch + sequential + 10),
                     # the run measures the kubelet's own CPU and startup latency, not the default
                     # 5-QPS API client / registry throttles
                     "--kube-api-qps", "100", "--kube-api-burst", "200", "--registry-qps", "0"] + rt_args,
                    tmp, "kubelet")
        procs.append(kl)
        plugin = None
        if gpu_pods:
            plugin = _spawn(["kubernetes_amd.cmd.device_plugin", "--plugins-dir",
                             os.path.join(tmp, "kubelet", "device-plugin", "plugins")], tmp, "device-plugin")
            procs.append(plugin)
        c = Client(url)
        t = time.time()
        while True:
            nodes = (await c.list("nodes"))["items"]
            if nodes and any(x.get("type") == "Ready" and x.get("status") == "True"
                             for x in nodes[0]["status"].get("conditions") or ()):
                if not gpu_pods or int((nodes[0]["status"].get("capacity") or {}).get("amd.com/gpu", "0")) >= 1:
                    break
            if time.time() - t > 90:
                raise TimeoutError("kubelet did not register" + (" its GPUs" if nodes else ""))
            await asyncio.sleep(0.1)
        sampler = Sampler(kl.pid, period).start()
        rts = Sampler(rt_proc.pid, period).start() if rt_proc is not None else None
        cpu0 = sampler.cpu_seconds()
        ns = "density"
        await c.create("namespaces", {"metadata": {"name": ns}})
        # batch: all at once
        names = [f"batch-{i}" for i in range(batch)]
        created = {}
        t0 = time.monotonic()
        for n in names:
            created[n] = time.monotonic()
            await c.create("pods", _pod(n), ns)
        seen = await _wait_running(c, ns, names, timeout)
        batch_lat = [seen[n] - created[n] for n in names if n in seen]
        batch_all = max(seen[n] for n in names) - t0 if len(seen) >= len(names) else float("inf")
        # background pods, then sequential creations
        bg = [f"bg-{i}" for i in range(background)]
        for n in bg:
            await c.create("pods", _pod(n), ns)
        await _wait_running(c, ns, bg, timeout)
        seq_lat = []
        for i in range(sequential):
            n = f"seq-{i}"
            t1 = time.monotonic()
            await c.create("pods", _pod(n), ns)
            s2 = await _wait_running(c, ns, [n], timeout)
            if n in s2:
                seq_lat.append(s2[n] - t1)
        cpu_per_pod = (sampler.cpu_seconds() - cpu0) / max(1, batch + background + sequential)
        gpu = await _gpu_phase(c, ns, gpu_pods, timeout) if gpu_pods else None
        await asyncio.sleep(period)        # the sample covering the last start
        cpu = sorted(sampler.cpu) or [0.0]
        rss = max(sampler.rss or [0])
        rt_cpu = sorted(rts.cpu) if rts is not None else None
        rt_rss = max(rts.rss or [0]) if rts is not None else None
        # steady state: every pod running, nothing changing
        await asyncio.sleep(settle)
        sampler.reset()
        await asyncio.sleep(monitor)
        sampler.stop()
        if rts is not None:
            rts.stop()
        steady = sorted(sampler.cpu) or [0.0]
        await c.close()
        out = {
            "batch": {"pods": batch, "p50_s": round(pct(batch_lat, .5), 3), "p90_s": round(pct(batch_lat, .9), 3),
                      "p99_s": round(pct(batch_lat, .99), 3), "all_running_s": round(batch_all, 3)},
            "sequential": {"pods": sequential, "background": background, "p50_s": round(pct(seq_lat, .5), 3),
                           "p90_s": round(pct(seq_lat, .9), 3), "p99_s": round(pct(seq_lat, .99), 3)},
            "kubelet_cpu_cores": {"p50": round(pct(cpu, .5), 3), "p95": round(pct(cpu, .95), 3)},
            "kubelet_rss_mib": round(rss / 2**20, 1),
            "kubelet_cpu_s_per_pod": round(cpu_per_pod, 4),
            "steady": {"pods": batch + background + sequential, "monitor_s": monitor,
                       "kubelet_cpu_cores": {"p50": round(pct(steady, .5), 3), "p95": round(pct(steady, .95), 3)},
                       "kubelet_rss_mib": round(max(sampler.rss or [0]) / 2**20, 1)},
            "runtime": runtime,
            "thresholds": THRESHOLDS,
        }
        if gpu is not None:
            out["gpu"] = gpu
        if rt_cpu is not None:
            rt_cpu = rt_cpu or [0.0]
            out["runtime_cpu_cores"] = {"p50": round(pct(rt_cpu, .5), 3), "p95": round(pct(rt_cpu, .95), 3)}
            out["runtime_rss_mib"] = round(rt_rss / 2**20, 1)
        out["within_thresholds"] = (
            out["batch"]["p50_s"] <= THRESHOLDS["batch"]["p50"] and out["batch"]["p99_s"] <= THRESHOLDS["batch"]["p99"]
            and out["batch"]["all_running_s"] <= THRESHOLDS["batch"]["all"]
            and out["sequential"]["p99_s"] <= THRESHOLDS["sequential"]["p99"]
            and out["kubelet_cpu_cores"]["p50"] <= THRESHOLDS["kubelet_cpu"]["p50"]
            and out["kubelet_cpu_cores"]["p95"] <= THRESHOLDS["kubelet_cpu"]["p95"]
            and out["kubelet_rss_mib"] <= THRESHOLDS["kubelet_rss_mib"]
            and out["steady"]["kubelet_cpu_cores"]["p95"] <= THRESHOLDS["steady_kubelet_cpu"]["p95"]
            and out["steady"]["kubelet_rss_mib"] <= THRESHOLDS["steady_kubelet_rss_mib"]
            and (rt_cpu is None or (out["runtime_cpu_cores"]["p95"] <= THRESHOLDS["runtime_cpu"]["p95"]
                                    and out["runtime_rss_mib"] <= THRESHOLDS["runtime_rss_mib"]))
            and (gpu is None or (not gpu["failed"]
                                 and gpu["sequential"]["running_p99_s"] <= THRESHOLDS["sequential"]["p99"])))
        return out
    finally:
        # the kubelet leaves containers running when it stops (by design: a restarted kubelet
        # adopts them), so the pods go first and the kubelet kills their containers
        try:
            if url is not None:
                await asyncio.wait_for(_drain_pods(url), 60)
        except Exception:          # noqa: BLE001 - best effort; the processes are stopped anyway
            pass
        for p in procs:
            p.terminate()
        for p in procs:
            try:
                p.wait(10)
            except subprocess.TimeoutExpired:
                p.kill()


def main(argv=None):
    ap = argparse.ArgumentParser("node-density")
    ap.add_argument("--batch", type=int, default=10)
    ap.add_argument("--sequential", type=int, default=10)
    ap.add_argument("--background", type=int, default=50)
    ap.add_argument("--monitor", type=float, default=10.0, help="steady-state monitoring seconds")
    ap.add_argument("--period", type=float, default=1.0, help="CPU/RSS sampling period (cAdvisor housekeeping)")
    ap.add_argument("--runtime", default="process", choices=["process", "remote"],
                    help="remote: kubelet -> CRI -> a separate kamd-cri process (tracked as the runtime)")
    ap.add_argument("--gpu-pods", type=int, default=0,
                    help="run N single-GPU HIP vector_add pods through the real amd.com/gpu plugin (needs a GPU)")
    a = ap.parse_args(argv)
    print(json.dumps(asyncio.run(run(a.batch, a.sequential, a.background, monitor=a.monitor, period=a.period,
                                     runtime=a.runtime, gpu_pods=a.gpu_pods))))


if __name__ == "__main__":
    main()
