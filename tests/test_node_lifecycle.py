"""Node lifecycle controller: zone states, rate-limited eviction queues, disruption modes, the
NoExecute taint manager, condition taints and deprecated taint keys.

Parity: `pkg/controller/node/nodecontroller_test.go` (TestMonitorNodeStatusEvictPods,
TestPodStatusChange, TestMonitorNodeStatusEvictPodsWithDisruption — zone states and rate
limiters), `pkg/controller/node/scheduler/rate_limited_queue_test.go`,
`taint_controller_test.go` (TestCreatePod / TestUpdateNode: immediate vs delayed eviction,
cancellation when taints go away).
"""
import asyncio

from kubernetes_amd.api import core
from kubernetes_amd.cluster import LocalCluster
from kubernetes_amd.controllers import nodelifecycle as nl


class Clock:
    def __init__(self):
        self.t = 1000.0

    def __call__(self):
        return self.t


def test_compute_zone_state_thresholds():
    r = lambda s: {"type": "Ready", "status": s}  # noqa: E731
    assert nl.compute_zone_state([r("True")] * 3) == (0, nl.NORMAL)
    assert nl.compute_zone_state([r("Unknown")] * 2) == (2, nl.FULL)
    # 2 of 3 not ready: not more than 2 -> still Normal (the reference needs > 2 unhealthy nodes)
    assert nl.compute_zone_state([r("True"), r("False"), r("Unknown")]) == (2, nl.NORMAL)
    assert nl.compute_zone_state([r("True")] + [r("Unknown")] * 3) == (3, nl.PARTIAL)
    assert nl.compute_zone_state([r("True")] * 3 + [r("Unknown")] * 3) == (3, nl.NORMAL)      # 0.5 < 0.55
    assert nl.compute_zone_state([r("True")] * 3 + [r("Unknown")] * 3, 0.5)[1] == nl.PARTIAL
    assert nl.compute_zone_state([r("True")] * 4 + [r("Unknown")] * 3)[1] == nl.NORMAL      # 3/7 < 0.55
    assert nl.compute_zone_state([None, None]) == (2, nl.FULL)


def test_rate_limited_timed_queue():
    clk = Clock()
    q = nl.RateLimitedTimedQueue(1.0, clk)          # 1 node/s, burst 1
    assert q.add("a") and q.add("b") and not q.add("a")
    done = []

    async def ok(v, uid):
        done.append(v)
        return True, 0.0

    async def go():
        await q.try_(ok)
        assert done == ["a"]                          # one token
        await q.try_(ok)
        assert done == ["a"]
        clk.t += 1.0
        await q.try_(ok)
        assert done == ["a", "b"]
        clk.t += 5
        await q.try_(ok)
        assert done == ["a", "b"] and not q.add("a")  # processed entries stay known ...
        assert q.remove("a") and q.add("a")            # ... until removed (node Ready again)
        q.swap_limiter(0)                              # stop evictions
        clk.t += 100
        await q.try_(ok)
        assert done == ["a", "b"]
        q.swap_limiter(10.0)
        clk.t += 1

        async def fail(v, uid):
            done.append("fail:" + v)
            return False, 2.0
        await q.try_(fail)
        assert done[-1] == "fail:a"
        clk.t += 1
        await q.try_(ok)
        assert done[-1] == "fail:a"                    # retried only after its wait
        clk.t += 1.5
        await q.try_(ok)
        assert done[-1] == "a"
    asyncio.run(go())


def test_min_toleration_and_matching():
    taints = [{"key": nl.UNREACHABLE_TAINT, "effect": "NoExecute"}]
    tol = {"key": nl.UNREACHABLE_TAINT, "operator": "Exists", "effect": "NoExecute"}
    ok, used = nl.matching_tolerations(taints, [dict(tol, tolerationSeconds=30), dict(tol, tolerationSeconds=10)])
    assert ok and nl.min_toleration_time(used) == 10
    ok, used = nl.matching_tolerations(taints, [tol])
    assert ok and nl.min_toleration_time(used) is None                 # forever
    assert nl.matching_tolerations(taints + [{"key": "x", "effect": "NoExecute"}], [tol])[0] is False
    assert nl.min_toleration_time([dict(tol, tolerationSeconds=-1)]) == 0


def _ctl(**kw):
    c = nl.NodeLifecycleController(None, None, recorder=_Rec(), clock=Clock(), **kw)
    return c


class _Rec:
    def event(self, *a, **k):
        pass


def _node(name, zone="z1"):
    return {"metadata": {"name": name, "labels": {nl.ZONE_LABEL: zone}}}


def test_disruption_modes_swap_limiters():
    """handleDisruption: Partial in a small cluster stops evictions, Full everywhere stops them
    and cancels queued ones, leaving master-disruption mode restores the normal rate."""
    c = _ctl(eviction_rate=0.1, secondary_eviction_rate=0.01, large_cluster_threshold=3)
    ready = {"type": "Ready", "status": "True"}
    down = {"type": "Ready", "status": "Unknown"}
    nodes = [_node(f"n{i}") for i in range(4)] + [_node("m0", "z2")]
    zone = nl.zone_key(nodes[0])

    async def go():
        await c._handle_disruption({zone: [ready] * 4, nl.zone_key(nodes[4]): [ready]}, nodes)
        assert c.zone_states[zone] == nl.NORMAL and c._queue_for(zone).qps == 0.1
        # 3 of 4 down, zone of 4 > threshold 3: secondary rate
        await c._handle_disruption({zone: [ready] + [down] * 3, nl.zone_key(nodes[4]): [ready]}, nodes)
        assert c.zone_states[zone] == nl.PARTIAL and c._queue_for(zone).qps == 0.01
        c.large_cluster = 50
        c.zone_states[zone] = nl.NORMAL
        await c._handle_disruption({zone: [ready] + [down] * 3, nl.zone_key(nodes[4]): [ready]}, nodes)
        assert c._queue_for(zone).qps == 0                         # small cluster: stop
        # every zone fully disrupted: master disruption mode, queued evictions cancelled
        c._queue_for(zone).add("n1")
        await c._handle_disruption({zone: [down] * 4, nl.zone_key(nodes[4]): [down]}, nodes)
        assert all(s == nl.FULL for s in c.zone_states.values())
        assert all(q.qps == 0 for q in c.zone_queues.values()) and not c._queue_for(zone).queued()
        # one zone back: exit the mode, probe timestamps reset, per-zone rates restored
        c.status = {"n0": {"ready": None, "probe": 0, "transition": 0}}
        await c._handle_disruption({zone: [down] * 4, nl.zone_key(nodes[4]): [ready]}, nodes)
        assert c.zone_states[zone] == nl.FULL and c._queue_for(zone).qps == 0.1   # Full -> normal rate
        assert c.zone_states[nl.zone_key(nodes[4])] == nl.NORMAL
        assert c.status["n0"]["probe"] == c.clock()
    asyncio.run(go())


async def _kill_kubelet(cl, name):
    """The node's kubelet dies: no heartbeats, no pod status writes."""
    await [n for n in cl.nodes if n.name == name][0].kubelet.stop()


def test_eviction_mode_deletes_pods_but_not_daemonset_pods(run):
    """1.9 default (TaintBasedEvictions off): the node goes Unknown, pods are marked not ready,
    then after pod_eviction_timeout the eviction queue deletes its pods (reason NodeLost)
    except DaemonSet-owned ones."""
    async def main():
        opts = {"nodelifecycle": {"monitor_period": 0.05, "grace": 0.3, "pod_eviction_timeout": 0.3,
                                  "eviction_rate": 50}}
        async with LocalCluster(nodes=2, gpus_per_node=2, controllers=["nodelifecycle"], controller_options=opts) as cl:
            c = cl.client
            target = cl.nodes[0].name
            # a finalizer keeps the evicted pod readable (the stub kubelet still finalizes deletions)
            await c.create("pods", {"metadata": {"name": "g", "namespace": "default", "finalizers": ["test/keep"]}, "spec": {
                "nodeSelector": {"kubernetes.io/hostname": target}, "containers": [{"name": "c", "image": "x", "resources": {"limits": {core.AMD_GPU: "1"}}}]}})
            await c.create("pods", {"metadata": {"name": "ds-pod", "namespace": "default", "ownerReferences": [
                {"apiVersion": "apps/v1", "kind": "DaemonSet", "name": "d", "uid": "u1", "controller": True}]},
                "spec": {"nodeName": target, "containers": [{"name": "c", "image": "x"}]}})
            await cl.wait_pod("g")
            await cl.wait_pod("ds-pod")
            await _kill_kubelet(cl, target)

            async def evicted():
                p = await c.get("pods", "g", "default")
                return p if p["metadata"].get("deletionTimestamp") else None
            p = await cl.wait_for(evicted, timeout=20)
            assert p["status"].get("reason") == "NodeLost"
            ready = core.get_condition(p["status"], "Ready")
            assert ready is None or ready["status"] == "False"
            ds = await c.get("pods", "ds-pod", "default")
            assert not ds["metadata"].get("deletionTimestamp")
            n = await c.get("nodes", target)
            assert core.get_condition(n["status"], "Ready")["status"] == "Unknown"
            assert not any(t["key"] == nl.UNREACHABLE_TAINT for t in n["spec"].get("taints") or [])
            events = (await c.list("events", "default"))["items"]
            assert any(e["reason"] == "NodeControllerEviction" for e in events)
            await c.patch("pods", "g", {"metadata": {"finalizers": None}}, "default")
    run(main(), timeout=60)


def test_all_nodes_down_is_master_disruption_no_evictions(run):
    async def main():
        opts = {"nodelifecycle": {"monitor_period": 0.05, "grace": 0.3, "pod_eviction_timeout": 0.2,
                                  "eviction_rate": 50}}
        async with LocalCluster(nodes=2, gpus_per_node=0, controllers=["nodelifecycle"], controller_options=opts) as cl:
            c = cl.client
            await c.create("pods", {"metadata": {"name": "p", "namespace": "default"}, "spec": {
                "nodeName": cl.nodes[0].name, "containers": [{"name": "c", "image": "x"}]}})
            await cl.wait_pod("p")
            for n in cl.nodes:
                await _kill_kubelet(cl, n.name)

            async def all_unknown():
                ns = (await c.list("nodes"))["items"]
                return all(core.get_condition(n["status"], "Ready")["status"] == "Unknown" for n in ns)
            await cl.wait_for(all_unknown, timeout=20)
            await asyncio.sleep(1.0)                 # well past pod_eviction_timeout
            p = await c.get("pods", "p", "default")
            assert not p["metadata"].get("deletionTimestamp")
            ctl = next(x for x in cl.cm.controllers if x.name == "nodelifecycle")
            assert set(ctl.zone_states.values()) == {nl.FULL}
    run(main(), timeout=60)


def test_taint_manager_deletes_untolerated_now_tolerated_later_and_cancels(run):
    async def main():
        opts = {"nodelifecycle": {"monitor_period": 0.05}}
        async with LocalCluster(nodes=1, gpus_per_node=0, controllers=["nodelifecycle"], controller_options=opts) as cl:
            c = cl.client
            node = cl.nodes[0].name
            tol = {"key": "maint", "operator": "Exists", "effect": "NoExecute"}
            for name, tols in (("plain", []), ("short", [dict(tol, tolerationSeconds=1)]), ("forever", [tol])):
                await c.create("pods", {"metadata": {"name": name, "namespace": "default"}, "spec": {
                    "nodeName": node, "tolerations": tols, "containers": [{"name": "c", "image": "x"}]}})
                await cl.wait_pod(name)
            await c.patch("nodes", node, {"spec": {"taints": [{"key": "maint", "effect": "NoExecute"}]}})

            async def deleting(name):
                try:
                    p = await c.get("pods", name, "default")
                except Exception:  # noqa: BLE001 - already gone
                    return True
                return bool(p["metadata"].get("deletionTimestamp"))
            await cl.wait_for(lambda: deleting("plain"), timeout=10)
            assert not await deleting("short")
            await cl.wait_for(lambda: deleting("short"), timeout=10)
            await asyncio.sleep(0.3)
            assert not await deleting("forever")
            # a scheduled deletion is cancelled when the taint goes away
            await c.create("pods", {"metadata": {"name": "late", "namespace": "default"}, "spec": {
                "nodeName": node, "tolerations": [dict(tol, tolerationSeconds=2)], "containers": [{"name": "c", "image": "x"}]}})
            ctl = next(x for x in cl.cm.controllers if x.name == "nodelifecycle")
            await cl.wait_for(lambda: asyncio.sleep(0, "default/late" in ctl.scheduled), timeout=10)
            await c.patch("nodes", node, {"spec": {"taints": None}})
            await cl.wait_for(lambda: asyncio.sleep(0, "default/late" not in ctl.scheduled), timeout=10)
            await asyncio.sleep(2.3)
            assert not await deleting("late")
    run(main(), timeout=60)


def test_condition_taints_and_deprecated_keys(run):
    async def main():
        opts = {"nodelifecycle": {"monitor_period": 0.05, "taint_nodes_by_condition": True}}
        async with LocalCluster(nodes=1, gpus_per_node=0, controllers=["nodelifecycle"], controller_options=opts) as cl:
            c = cl.client
            node = cl.nodes[0].name
            await _kill_kubelet(cl, node)    # the kubelet would rewrite the conditions patched below
            await c.patch("nodes", node, {"spec": {"taints": [
                {"key": "node.alpha.kubernetes.io/notReady", "effect": "NoSchedule"}]}})

            async def fixed():
                n = await c.get("nodes", node)
                keys = [t["key"] for t in n["spec"].get("taints") or []]
                return keys == [nl.NOT_READY_TAINT]
            await cl.wait_for(fixed, timeout=10)
            n = await c.get("nodes", node)
            conds = [dict(x) for x in n["status"]["conditions"]]
            for x in conds:
                if x["type"] == "MemoryPressure":
                    x["status"] = "True"
            await c.patch("nodes", node, {"status": {"conditions": conds}}, None, "merge", "status")

            async def mem_taint():
                n = await c.get("nodes", node)
                return any(t["key"] == "node.kubernetes.io/memory-pressure" and t["effect"] == "NoSchedule"
                           for t in n["spec"].get("taints") or [])
            await cl.wait_for(mem_taint, timeout=10)
    run(main(), timeout=60)
