"""Scheduler: ER allocation (fork F4/F5 tests `extended_resources_test.go:59-193`,
`node_info_test.go`), topology-aware placement, the assume fix, end-to-end with the API server."""
import asyncio
import os

import pytest

from kubernetes_amd.api import core
from kubernetes_amd.apiserver.server import APIServer
from kubernetes_amd.client.rest import Client
from kubernetes_amd.scheduler.cache import ERManager, NodeInfo, PodInfo, SchedulerCache
from kubernetes_amd.scheduler.generic import FitError, GenericScheduler
from kubernetes_amd.scheduler.scheduler import Scheduler
from kubernetes_amd.scheduler.topology import REQUIRED, Request, allocate


def gpu_dev(i, hive="h0", numa="0", mem="294912", health=core.HEALTHY, links="7", arch="gfx950"):
    return {"id": f"g{i}", "health": health, "attributes": {
        core.ATTR_INDEX: str(i), core.ATTR_HIVE: hive, core.ATTR_NUMA: numa, core.ATTR_MEMORY: mem,
        core.ATTR_HBM: f"{int(mem) // 1024}Gi", core.ATTR_XGMI_LINKS: links, core.ATTR_ARCH: arch}}


def node(name, devs, cpu="64", mem="512Gi", labels=None, taints=None):
    return {"metadata": {"name": name, "labels": labels or {}},
            "spec": {"taints": taints or []},
            "status": {"allocatable": {"cpu": cpu, "memory": mem, "pods": "110"},
                       "conditions": [{"type": "Ready", "status": "True"}],
                       "extendedResources": {core.AMD_GPU: {"resources": {d["id"]: d for d in devs}}}}}


def gpu_pod(name, n, required=None, annotations=None, ns="default"):
    return {"metadata": {"name": name, "namespace": ns, "uid": "uid-" + name, "annotations": annotations or {}},
            "spec": {"containers": [{"name": "c", "image": "x", "extendedResourceRequests": ["er"]}],
                     "extendedResources": [{"name": "er", "resources": {"limits": {core.AMD_GPU: str(n)},
                                                                        "requests": {core.AMD_GPU: str(n)}},
                                            "affinity": {"required": required or []}}]}}


def er_of(devs):
    e = ERManager()
    e.set_node(node("n", devs))
    return e


def test_selectors_gt_lt_in_and_quantities():
    devs = [gpu_dev(0, mem="8000"), gpu_dev(1, mem="294912"), gpu_dev(2, mem="294912", arch="gfx942")]
    e = er_of(devs)
    r = Request("er", core.AMD_GPU, 1, [{"key": core.ATTR_MEMORY, "operator": "Gt", "values": ["100000"]},
                                        {"key": core.ATTR_ARCH, "operator": "In", "values": ["gfx950"]}])
    b, _, _ = allocate([r], e)
    assert b == {"er": {"resources": ["g1"]}}
    # quantity-aware: hbm > 256Gi
    r = Request("er", core.AMD_GPU, 2, [{"key": core.ATTR_HBM, "operator": "Gt", "values": ["256Gi"]}])
    b, _, _ = allocate([r], e)
    assert sorted(b["er"]["resources"]) == ["g1", "g2"]
    r = Request("er", core.AMD_GPU, 1, [{"key": core.ATTR_MEMORY, "operator": "Lt", "values": ["9000"]}])
    assert allocate([r], e)[0] == {"er": {"resources": ["g0"]}}
    r = Request("er", core.AMD_GPU, 3, [{"key": core.ATTR_MEMORY, "operator": "Gt", "values": ["100000"]}])
    b, _, why = allocate([r], e)
    assert b is None and "Insufficient" in why


def test_unhealthy_devices_not_allocated():
    e = er_of([gpu_dev(0, health=core.UNHEALTHY), gpu_dev(1)])
    b, _, _ = allocate([Request("er", core.AMD_GPU, 1, [])], e)
    assert b == {"er": {"resources": ["g1"]}}
    assert allocate([Request("er", core.AMD_GPU, 2, [])], e)[0] is None


def test_hive_and_numa_aware_multi_gpu():
    # two hives of 4; hive h1 has only 3 free -> a 4-GPU pod must take h0 entirely
    devs = [gpu_dev(i, hive="h0" if i < 4 else "h1", numa="0" if i < 4 else "1") for i in range(8)]
    e = er_of(devs)
    e.add_pod("x/y", {core.AMD_GPU: ["g7"]})
    b, score, _ = allocate([Request("er", core.AMD_GPU, 4, [])], e)
    assert sorted(b["er"]["resources"]) == ["g0", "g1", "g2", "g3"]
    # a 2-GPU pod best-fits into the partially used hive h1
    b, _, _ = allocate([Request("er", core.AMD_GPU, 2, [])], e)
    assert sorted(b["er"]["resources"]) == ["g4", "g5"]
    # 5 GPUs: no hive fits; preferred spans, required fails
    b, s, _ = allocate([Request("er", core.AMD_GPU, 5, [])], e)
    assert b is not None and len(b["er"]["resources"]) == 5 and s <= 1
    b, _, why = allocate([Request("er", core.AMD_GPU, 5, [])], e, REQUIRED)
    assert b is None and "hive" in why


def test_single_gpu_packs_used_hive_first():
    devs = [gpu_dev(i, hive="h0" if i < 4 else "h1") for i in range(8)]
    e = er_of(devs)
    e.add_pod("a/b", {core.AMD_GPU: ["g0"]})
    b, _, _ = allocate([Request("er", core.AMD_GPU, 1, [])], e)
    assert b["er"]["resources"] == ["g1"]


def test_link_health_gates_multi_gpu():
    devs = [gpu_dev(i, links="7" if i != 2 else "1") for i in range(4)]
    e = er_of(devs)
    b, _, _ = allocate([Request("er", core.AMD_GPU, 4, [])], e)
    assert b is None
    b, _, _ = allocate([Request("er", core.AMD_GPU, 3, [])], e)
    assert sorted(b["er"]["resources"]) == ["g0", "g1", "g3"]


def test_assume_reserves_devices_binpack_8_single_gpu_pods():
    """BASELINE config 3: 8 single-GPU pods on one 8-GPU node, back to back before any bind
    completes — every pod must get a distinct device (the reference could double-assign)."""
    cache = SchedulerCache()
    cache.add_node(node("mi355x-0", [gpu_dev(i) for i in range(8)]))
    gs = GenericScheduler(cache)
    got = []
    for i in range(8):
        p = gpu_pod(f"p{i}", 1)
        host, erb = gs.schedule(p)
        assumed = dict(p, spec=dict(p["spec"], nodeName=host,
                                    extendedResources=[dict(p["spec"]["extendedResources"][0], assigned=erb["er"]["resources"])]))
        cache.assume_pod(assumed)
        got.extend(erb["er"]["resources"])
    assert sorted(got) == [f"g{i}" for i in range(8)]
    with pytest.raises(FitError) as ei:
        gs.schedule(gpu_pod("p9", 1))
    assert "Insufficient amd.com/gpu" in str(ei.value)


def test_predicates_taints_selector_resources():
    cache = SchedulerCache()
    cache.add_node(node("a", [gpu_dev(0)], labels={"zone": "z1"},
                        taints=[{"key": core.AMD_GPU, "effect": "NoSchedule"}]))
    cache.add_node(node("b", [gpu_dev(0)], cpu="1", labels={"zone": "z2"}))
    gs = GenericScheduler(cache)
    p = gpu_pod("p", 1)
    p["spec"]["containers"][0]["resources"] = {"requests": {"cpu": "2"}}
    with pytest.raises(FitError) as ei:
        gs.schedule(p)
    msg = str(ei.value)
    assert "taints" in msg and "Insufficient cpu" in msg
    p["spec"]["tolerations"] = [{"key": core.AMD_GPU, "operator": "Exists", "effect": "NoSchedule"}]
    assert gs.schedule(p)[0] == "a"
    p2 = gpu_pod("q", 1)
    p2["spec"]["nodeSelector"] = {"zone": "z2"}
    assert gs.schedule(p2)[0] == "b"


def test_gpu_binpacking_prefers_fuller_node():
    cache = SchedulerCache()
    cache.add_node(node("empty", [gpu_dev(i) for i in range(8)]))
    cache.add_node(node("half", [gpu_dev(i) for i in range(8)]))
    p0 = gpu_pod("x", 4)
    p0["spec"]["nodeName"] = "half"
    p0["spec"]["extendedResources"][0]["assigned"] = ["g0", "g1", "g2", "g3"]
    cache.add_pod(p0)
    gs = GenericScheduler(cache)
    assert gs.schedule(gpu_pod("y", 4))[0] == "half"
    assert gs.schedule(gpu_pod("z", 8))[0] == "empty"


def test_end_to_end_scheduler_binds_distinct_devices(run):
    async def main():
        s = APIServer()
        port = await s.start()
        c = Client(f"http://127.0.0.1:{port}")
        await c.create("nodes", node("mi355x-0", [gpu_dev(i) for i in range(8)]))
        await c.update_status("nodes", node("mi355x-0", [gpu_dev(i) for i in range(8)]) | {"metadata": (await c.get("nodes", "mi355x-0"))["metadata"]})
        sched = Scheduler(Client(f"http://127.0.0.1:{port}"))
        task = asyncio.ensure_future(sched.run())
        for i in range(8):
            await c.create("pods", {"metadata": {"name": f"p{i}", "namespace": "default"},
                                    "spec": {"containers": [{"name": "c", "image": "x",
                                                             "resources": {"limits": {core.AMD_GPU: "1"}}}]}})
        await c.create("pods", {"metadata": {"name": "big", "namespace": "default"},
                                "spec": {"containers": [{"name": "c", "image": "x",
                                                         "resources": {"limits": {core.AMD_GPU: "4"}}}]}})
        for _ in range(200):
            pods = (await c.list("pods", "default"))["items"]
            bound = [p for p in pods if p["spec"].get("nodeName")]
            if len(bound) == 8:
                break
            await asyncio.sleep(0.02)
        ids = [i for p in bound for i in p["spec"]["extendedResources"][0]["assigned"]]
        assert len(bound) == 8 and len(set(ids)) == 8
        big = await c.get("pods", "big", "default")
        assert not big["spec"].get("nodeName")
        # free 4 GPUs -> the 4-GPU pod schedules
        for i in range(4):
            await c.delete("pods", f"p{i}", "default", grace_period=0)
        for _ in range(200):
            big = await c.get("pods", "big", "default")
            if big["spec"].get("nodeName"):
                break
            await asyncio.sleep(0.02)
        assert len(big["spec"]["extendedResources"][0]["assigned"]) == 4
        cond = core.get_condition(big["status"], core.COND_POD_SCHEDULED)
        assert cond["status"] == "True"
        evs = (await c.list("events", "default"))["items"]
        assert any(e["reason"] == "FailedScheduling" for e in evs)
        task.cancel()
        await sched.stop()
        await c.close()
        await s.stop()
    run(main())


def test_equivalence_cache_matches_uncached_decisions():
    """The equivalence cache must not change any decision (equivalence_cache.go contract)."""
    import random
    rng = random.Random(7)
    caches = [SchedulerCache(), SchedulerCache()]
    for c in caches:
        for k in range(6):
            c.add_node(node(f"n{k}", [gpu_dev(i, hive="h0" if i < 4 else "h1", numa=str(i // 4)) for i in range(8)],
                            cpu=str(8 + k), labels={"zone": f"z{k % 2}"}))
    scheds = [GenericScheduler(caches[0], equivalence_cache=True), GenericScheduler(caches[1], equivalence_cache=False)]
    live = []
    for step in range(300):
        if live and rng.random() < 0.35:
            victim = live.pop(rng.randrange(len(live)))
            for c in caches:
                c.remove_pod(victim)
            continue
        n = rng.choice([1, 1, 1, 2, 4])
        p = gpu_pod(f"p{step}", n)
        p["spec"]["containers"][0]["resources"] = {"requests": {"cpu": rng.choice(["500m", "1", "2"])}}
        if rng.random() < 0.2:
            p["spec"]["nodeSelector"] = {"zone": "z1"}
        out = []
        for s in scheds:
            try:
                out.append(s.schedule(p))
            except FitError as e:
                out.append(("fit", str(e)))
        assert out[0] == out[1], (step, out)
        if out[0][0] != "fit":
            host, erb = out[0]
            ap = dict(p, spec=dict(p["spec"], nodeName=host,
                                   extendedResources=[dict(p["spec"]["extendedResources"][0], assigned=erb["er"]["resources"])]))
            for c in caches:
                c.assume_pod(ap)
            live.append(ap)
    assert scheds[0].ecache_hits > 0


def _sharded_run(run, shared):
    """Two partitioned scheduler shards: each sees only its own unassigned pods and its own
    nodes' pods; pods that do not fit are handed to the other shard; nothing is double-assigned."""
    from kubernetes_amd.api.sharding import shard_of_key

    async def main():
        store = None
        if shared:
            from kubernetes_amd.storage.remote import StoreServer
            store = StoreServer()
            s = APIServer(store=store.start())
        else:
            s = APIServer()
        port = await s.start()
        c = Client(f"http://127.0.0.1:{port}")
        for name, n in (("a-node", 8), ("b-node", 1)):
            await c.create("nodes", node(name, [gpu_dev(i) for i in range(n)]))
            await c.update_status("nodes", node(name, [gpu_dev(i) for i in range(n)]) | {"metadata": (await c.get("nodes", name))["metadata"]})
        scheds = [Scheduler(Client(f"http://127.0.0.1:{port}"), shard_index=i, shard_count=2, rehandoff_period=0.3)
                  for i in range(2)]
        tasks = [asyncio.ensure_future(x.run()) for x in scheds]

        def pod(name):
            return {"metadata": {"name": name, "namespace": "default"},
                    "spec": {"containers": [{"name": "c", "image": "x", "resources": {"limits": {core.AMD_GPU: "1"}}}]}}
        names = [f"p{i}" for i in range(9)]
        assert sum(shard_of_key(f"default/{n}", 2) == 1 for n in names) >= 2   # b-node (1 GPU) overflows
        for n in names:
            await c.create("pods", pod(n))

        async def bound():
            return [p for p in (await c.list("pods", "default"))["items"] if p["spec"].get("nodeName")]
        for _ in range(300):
            b = await bound()
            if len(b) == 9:
                break
            await asyncio.sleep(0.02)
        ids = [(p["spec"]["nodeName"], i) for p in b for i in p["spec"]["extendedResources"][0]["assigned"]]
        assert len(b) == 9 and len(set(ids)) == 9
        assert sum(x.handoffs for x in scheds) >= 1
        assert set(scheds[0].owned) == {"a-node"} and set(scheds[1].owned) == {"b-node"}
        assert all(n in scheds[0].cache.nodes for n in ("a-node",)) and "b-node" not in scheds[0].cache.nodes
        # cluster full: the 10th pod goes round both shards and is reported unschedulable
        await c.create("pods", pod("late"))
        for _ in range(300):
            evs = (await c.list("events", "default"))["items"]
            if any(e["reason"] == "FailedScheduling" and e["involvedObject"]["name"] == "late" for e in evs):
                break
            await asyncio.sleep(0.02)
        else:
            raise AssertionError("no FailedScheduling for the overflow pod")
        # capacity frees on either node: the pod is picked up (same shard or re-offered)
        victim = next(p for p in b if p["spec"]["nodeName"] == "b-node")
        await c.delete("pods", victim["metadata"]["name"], "default", grace_period=0)
        for _ in range(300):
            late = await c.get("pods", "late", "default")
            if late["spec"].get("nodeName"):
                break
            await asyncio.sleep(0.02)
        assert late["spec"].get("nodeName") == "b-node"
        for t in tasks:
            t.cancel()
        for x in scheds:
            await x.stop()
        await c.close()
        await s.stop()
        if store is not None:
            store.stop()
    run(main())


def test_partitioned_scheduler_shards_embedded(run):
    _sharded_run(run, shared=False)


def test_partitioned_scheduler_shards_shared_store_fanout(run):
    _sharded_run(run, shared=True)


# -- compute partitions (CPX/QPX): logical devices that share an MI355X package ----------------

def cpx_devs(sockets=2, per=8, part="CPX", hive="h0", links="7"):
    """Device entries as the amd.com/gpu plugin advertises them for a CPX node (fixture-built)."""
    from kubernetes_amd.deviceplugin.amdgpu import gpu_attributes
    from kubernetes_amd.native import amdsmi
    if not os.path.exists(amdsmi.lib_path()):
        out = []
        for s in range(sockets):
            for p in range(per):
                d = gpu_dev(s * per + p, hive=hive, links=links)
                d["attributes"].update({core.ATTR_PARTITION: part, core.ATTR_SOCKET: str(s),
                                        core.ATTR_PARTITION_ID: str(p)})
                out.append(d)
        return out
    smi = amdsmi.SMI(fixture=amdsmi.fixture_file(sockets, partition=part, seed="cpx"))
    out = []
    for g in smi.gpus():
        a = gpu_attributes(g, smi.metrics(g.index))
        a[core.ATTR_HIVE] = hive
        a[core.ATTR_XGMI_LINKS] = links
        out.append({"id": f"g{g.index}", "health": core.HEALTHY, "attributes": a})
    return out


def _sockets(e, ids):
    return {e.available[core.AMD_GPU][i]["attributes"][core.ATTR_SOCKET] for i in ids}


def test_cpx_partitions_pack_into_one_package():
    devs = cpx_devs(2)
    assert {d["attributes"][core.ATTR_PARTITION] for d in devs} == {"CPX"} and len(devs) == 16
    e = er_of(devs)
    # 8 partitions = one whole package; with only 1 xGMI link up they still fit (no links used)
    b, score, _ = allocate([Request("er", core.AMD_GPU, 8, [])], er_of(cpx_devs(2, links="0")))
    assert b is not None and len(_sockets(e, b["er"]["resources"])) == 1 and score == 10.0
    # single partitions fill a package before opening the next one
    e.add_pod("a/b", {core.AMD_GPU: ["g0"]})
    b, _, _ = allocate([Request("er", core.AMD_GPU, 1, [])], e)
    assert b["er"]["resources"] == ["g1"]
    # a 4-partition pod fits in ONE package; the used one (6 free) is the best fit
    b, _, _ = allocate([Request("er", core.AMD_GPU, 4, [])], e)
    assert _sockets(e, b["er"]["resources"]) == {"0"}
    # 12 partitions: the whole free package + 4 of the used one (fewest packages)
    b, _, _ = allocate([Request("er", core.AMD_GPU, 12, [])], e)
    ids = b["er"]["resources"]
    assert len(ids) == 12 and len(_sockets(e, ids)) == 2 and "g0" not in ids


def test_cpx_multi_package_needs_links_per_package():
    # 16 partitions span 2 packages -> each needs >= 1 xGMI link
    assert allocate([Request("er", core.AMD_GPU, 16, [])], er_of(cpx_devs(2, links="0")))[0] is None
    b, _, _ = allocate([Request("er", core.AMD_GPU, 16, [])], er_of(cpx_devs(2, links="1")))
    assert b is not None and len(b["er"]["resources"]) == 16


def test_cpx_scheduler_prefers_node_with_partly_used_package():
    cache = SchedulerCache()
    cache.add_node(node("fresh", cpx_devs(2)))
    cache.add_node(node("used", cpx_devs(2)))
    p0 = gpu_pod("x", 3)
    p0["spec"]["nodeName"] = "used"
    p0["spec"]["extendedResources"][0]["assigned"] = ["g0", "g1", "g2"]
    cache.add_pod(p0)
    gs = GenericScheduler(cache)
    host, erb = gs.schedule(gpu_pod("y", 5))           # fills package 0 of "used" exactly
    assert host == "used" and sorted(erb["er"]["resources"]) == [f"g{i}" for i in range(3, 8)]
    # selector on the partition mode / per-partition compute units
    host, _ = gs.schedule(gpu_pod("z", 1, required=[{"key": core.ATTR_CUS, "operator": "Lt", "values": ["64"]}]))
    assert host in ("fresh", "used")
