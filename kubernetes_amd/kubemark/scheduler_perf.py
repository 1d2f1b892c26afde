"""scheduler_perf equivalent: scheduler throughput against fake nodes, no kubelets.

Parity: `test/integration/scheduler_perf/scheduler_test.go:34-182` and `util.go:31-80` — an API
server and the scheduler, Node objects written straight into the API (4 CPU / 32 Gi / 110 pods
in the reference), N pods created up front, and the number of scheduled pods sampled once per
second; the test fails if the WORST 1-s interval is below 30 pods/s (warns below 100).

Two workloads:
  * `cpu`  — the reference's: 100 nodes x (4 CPU, 32 Gi, 110 pods), 3000 pods with no requests.
  * `gpu`  — the MI355X one: nodes advertising 8 MI355X each (one xGMI hive, Node.status
             .extendedResources as the device plugin publishes it), 1-GPU pods through the ResourceV2
             admission and the device allocator. With `gpus_per_pod=4` the pods carry
             `amd.com/xgmi-policy: required` and must land inside one hive.

Scheduled = observed `spec.nodeName` on a pod watch (bind acknowledged by the API server).
"""
from __future__ import annotations

import asyncio
import time

from ..api import core
from ..client.rest import Client
from .density import interval_rates

FAIL_BELOW = 30.0    # scheduler_test.go:35
WARN_BELOW = 100.0   # scheduler_test.go:36


def fake_node(name, gpus=0, cpu="4", memory="32Gi", pods="110", hive="hive-0"):
    st = {"capacity": {"cpu": cpu, "memory": memory, "pods": pods},
          "allocatable": {"cpu": cpu, "memory": memory, "pods": pods},
          "conditions": [{"type": "Ready", "status": "True"}]}
    if gpus:
        devs = {}
        for i in range(gpus):
            did = f"{name}-GPU-{i}"
            devs[did] = {"id": did, "health": core.HEALTHY, "attributes": {
                core.ATTR_ARCH: "gfx950", core.ATTR_PRODUCT: "MI355X", core.ATTR_MEMORY: "294912",
                core.ATTR_HBM: "288Gi", core.ATTR_HIVE: f"{name}-{hive}", core.ATTR_NUMA: str(i // 4),
                core.ATTR_INDEX: str(i), core.ATTR_XGMI_LINKS: "7"}}
        st["extendedResources"] = {core.AMD_GPU: {"resources": devs}}
        st["capacity"][core.AMD_GPU] = str(gpus)
        st["allocatable"][core.AMD_GPU] = str(gpus)
    return {"apiVersion": "v1", "kind": "Node", "metadata": {"name": name, "labels": {"kubernetes.io/hostname": name}},
            "spec": {}, "status": st}


def perf_pod(name, ns, gpus=0):
    c = {"name": "c", "image": "kubernetes-amd/pause:1"}
    md = {"name": name, "namespace": ns, "labels": {"app": "scheduler-perf"}}
    if gpus:
        c["resources"] = {"limits": {core.AMD_GPU: str(gpus)}}
        if gpus > 1:
            md["annotations"] = {"amd.com/xgmi-policy": "required"}
    return {"apiVersion": "v1", "kind": "Pod", "metadata": md, "spec": {"containers": [c]}}


async def run_scheduler_perf(url, nodes=100, pods=3000, workload="cpu", gpus_per_node=8, gpus_per_pod=1,
                             namespace="sched-perf", create_concurrency=64, timeout=600.0):
    """Create nodes, then pods; return throughput stats. The scheduler must already be running."""
    c = Client(url, max_conns=create_concurrency)
    gpu = workload == "gpu"
    try:
        sem = asyncio.Semaphore(create_concurrency)

        async def mk_node(i):
            async with sem:
                n = fake_node(f"perf-node-{i}", gpus=gpus_per_node if gpu else 0)
                st = n.pop("status")
                created = await c.create("nodes", dict(n))
                created["status"] = st
                await c.update_status("nodes", created)
        await asyncio.gather(*(mk_node(i) for i in range(nodes)))
        try:
            await c.create("namespaces", {"metadata": {"name": namespace}})
        except Exception:
            pass
        # let the scheduler's node informer see every node before the clock starts
        await asyncio.sleep(1.0)
        lst = await c.list("pods", namespace)
        stream = await c.watch("pods", namespace, lst["metadata"]["resourceVersion"])
        scheduled: dict[str, float] = {}
        done = asyncio.Event()
        t0 = [None]

        async def watch():
            async for _, p in stream:
                if (p.get("spec") or {}).get("nodeName") and p["metadata"]["name"] not in scheduled:
                    scheduled[p["metadata"]["name"]] = time.monotonic()
                    if len(scheduled) >= pods:
                        done.set()
        wt = asyncio.ensure_future(watch())
        t0[0] = time.monotonic()

        async def mk_pod(i):
            async with sem:
                await c.create("pods", perf_pod(f"perf-pod-{i}", namespace, gpus_per_pod if gpu else 0), namespace)
        creator = asyncio.ensure_future(asyncio.gather(*(mk_pod(i) for i in range(pods))))
        try:
            await asyncio.wait_for(done.wait(), timeout)
        finally:
            stream.close()
            wt.cancel()
        await creator
        times = [t - t0[0] for t in scheduled.values()]
        avg, worst = interval_rates(times)
        elapsed = max(times) if times else float("nan")
        hive_ok = None
        if gpu and gpus_per_pod > 1:
            allp = (await c.list("pods", namespace))["items"]
            hive_ok = sum(1 for p in allp if len({a.rsplit("-GPU-", 1)[0] for a in
                                                   core.pod_assigned_devices(p).get(core.AMD_GPU, [])}) == 1)
        return {"workload": workload, "nodes": nodes, "pods": pods, "gpus_per_node": gpus_per_node if gpu else 0,
                "gpus_per_pod": gpus_per_pod if gpu else 0, "scheduled": len(scheduled),
                "elapsed_s": round(elapsed, 3), "throughput_pods_per_s": round(len(scheduled) / elapsed, 1),
                # a run shorter than one second has no full 1-s interval: its worst interval is
                # unmeasured (None), not the average
                "avg_interval_pods_per_s": round(avg, 1),
                "min_interval_pods_per_s": round(worst, 1) if worst is not None else None,
                "full_intervals": int(elapsed) if times else 0,
                "pass": (worst >= FAIL_BELOW) if worst is not None else None,
                "warn": (worst < WARN_BELOW) if worst is not None else None, "single_node_pods": hive_ok}
    finally:
        await c.close()
