"""scheduler_perf harness (small sizes): CPU and GPU workloads pass the reference's 30 pods/s bar,
every GPU pod gets distinct devices, 4-GPU pods stay on one node's hive."""
import asyncio

from kubernetes_amd.api import core
from kubernetes_amd.apiserver.server import APIServer
from kubernetes_amd.client.rest import Client
from kubernetes_amd.kubemark.scheduler_perf import run_scheduler_perf
from kubernetes_amd.scheduler.scheduler import Scheduler


def _run(run, **kw):
    async def main():
        s = APIServer()
        port = await s.start()
        url = f"http://127.0.0.1:{port}"
        sched = Scheduler(Client(url), emit_events=False)
        t = asyncio.ensure_future(sched.run())
        try:
            r = await run_scheduler_perf(url, timeout=120, **kw)
            pods = [e.obj for e in s.caches["pods"].by_key.values()]
            return r, pods
        finally:
            await sched.stop()
            t.cancel()
            await s.stop()
    return run(main())


def test_cpu_workload(run):
    r, _ = _run(run, nodes=20, pods=300, workload="cpu")
    assert r["scheduled"] == 300 and r["pass"] is not False and r["throughput_pods_per_s"] >= 30, r


def test_gpu_workload_distinct_devices(run):
    r, pods = _run(run, nodes=10, pods=80, workload="gpu", gpus_per_node=8)
    assert r["scheduled"] == 80 and r["pass"] is not False and r["throughput_pods_per_s"] >= 30, r
    seen = set()
    for p in pods:
        for i in core.pod_assigned_devices(p).get(core.AMD_GPU, []):
            assert i not in seen
            seen.add(i)
    assert len(seen) == 80            # the cluster is exactly full: 10 nodes x 8 GPUs


def test_gpu_4gpu_pods_single_node(run):
    r, pods = _run(run, nodes=4, pods=8, workload="gpu", gpus_per_node=8, gpus_per_pod=4)
    assert r["scheduled"] == 8 and r["single_node_pods"] == 8, r
