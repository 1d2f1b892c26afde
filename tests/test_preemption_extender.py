"""Priority preemption (GPU-aware victim selection) and HTTP scheduler extenders."""
import asyncio

from kubernetes_amd.api import core
from kubernetes_amd.cluster import LocalCluster
from kubernetes_amd.scheduler.cache import PodInfo, SchedulerCache
from kubernetes_amd.scheduler.extender import HTTPExtender
from kubernetes_amd.scheduler.generic import GenericScheduler
from kubernetes_amd.scheduler.preemption import preempt, select_victims
from kubernetes_amd.utils.httpserver import HTTPServer, Response

from test_scheduler import gpu_dev, gpu_pod, node


def bound(name, ids, prio=0, node_name="n0"):
    p = gpu_pod(name, len(ids))
    p["spec"]["nodeName"] = node_name
    p["spec"]["priority"] = prio
    p["spec"]["extendedResources"][0]["assigned"] = list(ids)
    return p


def test_victims_are_minimal_and_respect_hives():
    cache = SchedulerCache()
    # 2 hives x 4 GPUs; hive h0 holds 4 low pods, hive h1 holds 2 low pods + 2 mid pods
    devs = [gpu_dev(i, hive="h0" if i < 4 else "h1", links="3") for i in range(8)]
    cache.add_node(node("n0", devs))
    for i in range(4):
        cache.add_pod(bound(f"low{i}", [f"g{i}"], prio=0))
    cache.add_pod(bound("low4", ["g4"], prio=0))
    cache.add_pod(bound("low5", ["g5"], prio=0))
    cache.add_pod(bound("mid6", ["g6"], prio=50))
    cache.add_pod(bound("mid7", ["g7"], prio=50))
    gs = GenericScheduler(cache)
    hi = gpu_pod("hi", 2, annotations={"amd.com/xgmi-policy": "required"})
    hi["spec"]["priority"] = 100
    victims = select_victims(gs, hi, PodInfo(hi), cache.nodes["n0"])
    # two GPUs in ONE hive must be freed; the cheapest is two priority-0 pods, never the mid pods
    assert len(victims) == 2 and all(v["spec"]["priority"] == 0 for v in victims)
    hives = {("h0" if int(v["spec"]["extendedResources"][0]["assigned"][0][1:]) < 4 else "h1") for v in victims}
    assert len(hives) == 1
    # a priority-10 pod may not evict priority-50 pods, and 2 low pods suffice
    mid = gpu_pod("m", 2)
    mid["spec"]["priority"] = 10
    n, v, _ = preempt(gs, mid, PodInfo(mid))
    assert n == "n0" and len(v) == 2 and all(x["spec"]["priority"] == 0 for x in v)
    # an equal-priority pod preempts nothing
    same = gpu_pod("s", 1)
    same["spec"]["priority"] = 0
    assert preempt(gs, same, PodInfo(same)) == (None, [], [])


def test_preemption_end_to_end(run):
    async def main():
        async with LocalCluster(nodes=1, gpus_per_node=8) as cl:
            c = cl.client
            await c.create("priorityclasses", {"apiVersion": "scheduling.k8s.io/v1alpha1", "kind": "PriorityClass",
                                               "metadata": {"name": "high"}, "value": 1000})
            for i in range(8):
                await c.create("pods", {"metadata": {"name": f"low{i}"},
                                        "spec": {"containers": [{"name": "c", "image": "x",
                                                                 "resources": {"limits": {core.AMD_GPU: "1"}}}],
                                                 "terminationGracePeriodSeconds": 0}})
            for i in range(8):
                await cl.wait_pod(f"low{i}")
            await c.create("pods", {"metadata": {"name": "big"},
                                    "spec": {"priorityClassName": "high",
                                             "containers": [{"name": "c", "image": "x",
                                                             "resources": {"limits": {core.AMD_GPU: "4"}}}]}})
            p = await cl.wait_pod("big", timeout=30)
            assert p["spec"]["priority"] == 1000
            assert len(p["spec"]["extendedResources"][0]["assigned"]) == 4
            left = [x for x in (await c.list("pods", "default"))["items"] if x["metadata"]["name"].startswith("low")
                    and not x["metadata"].get("deletionTimestamp")]
            assert len(left) == 4
    run(main(), timeout=120)


def test_http_extender_filter_and_prioritize(run):
    calls = []

    async def handler(req):
        import json
        body = json.loads(req.body)
        names = body.get("nodenames") or [n["metadata"]["name"] for n in body["nodes"]["items"]]
        calls.append(req.path)
        if req.path.endswith("/filter"):
            keep = [n for n in names if n != "n1"]
            return Response(200, json.dumps({"nodenames": keep, "failedNodes": {"n1": "vetoed by extender"}}).encode())
        return Response(200, json.dumps([{"host": n, "score": 10 if n == "n2" else 0} for n in names]).encode())

    async def main():
        srv = HTTPServer(handler)
        port = await srv.start()
        try:
            ext = HTTPExtender(f"http://127.0.0.1:{port}/ext", "filter", "prioritize", weight=100,
                               node_cache_capable=True, managed_resources=[core.AMD_GPU])
            cache = SchedulerCache()
            for n in ("n0", "n1", "n2"):
                cache.add_node(node(n, [gpu_dev(i) for i in range(8)]))
            gs = GenericScheduler(cache, extenders=[ext])
            loop = asyncio.get_running_loop()
            host, _ = await loop.run_in_executor(None, gs.schedule, gpu_pod("p", 1))
            assert host == "n2"
            assert calls == ["/ext/filter", "/ext/prioritize"]
            # not interested in a CPU-only pod: no calls
            cpu_pod = {"metadata": {"name": "cpu", "namespace": "default"}, "spec": {"containers": [{"name": "c"}]}}
            await loop.run_in_executor(None, gs.schedule, cpu_pod)
            assert len(calls) == 2
        finally:
            await srv.stop()
    run(main())
