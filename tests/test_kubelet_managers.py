"""Kubelet managers: CPU manager static policy (GPU-NUMA aligned), eviction manager, static pods."""
import asyncio
import json
import os

import pytest

from kubernetes_amd.api import core
from kubernetes_amd.cluster import LocalCluster
from kubernetes_amd.kubelet.cpumanager import CPUTopology, StaticPolicy, format_cpulist, parse_cpulist, take_by_topology
from kubernetes_amd.kubelet.eviction import EvictionManager, parse_thresholds


def test_cpulist_roundtrip_and_topology_take():
    assert parse_cpulist("0-3,8,10-11") == [0, 1, 2, 3, 8, 10, 11]
    assert format_cpulist([11, 0, 1, 2, 3, 8, 10]) == "0-3,8,10-11"
    t = CPUTopology.synthetic(sockets=2, cores_per_socket=8, threads_per_core=2)
    # whole physical cores (hyperthread pairs) first
    assert take_by_topology(t, set(t.cpus), 4) == [0, 1, 16, 17]
    # a full socket when asked for one
    assert take_by_topology(t, set(t.cpus), 16) == list(range(0, 8)) + list(range(16, 24))
    # NUMA preference (GPUs on socket 1)
    assert {t.cpus[c].numa for c in take_by_topology(t, set(t.cpus), 6, prefer_numa=[1])} == {1}


def test_static_policy_exclusive_and_checkpoint(tmp_path):
    t = CPUTopology.synthetic(2, 4, 2)
    sf = str(tmp_path / "state")
    p = StaticPolicy(t, reserved=1, state_file=sf)
    assert len(p.shared_pool()) == 15
    g = {"metadata": {"uid": "u1"}, "status": {"qosClass": "Guaranteed"}}
    c = {"name": "c", "resources": {"requests": {"cpu": "4"}, "limits": {"cpu": "4"}}}
    cpus = p.allocate(g, c, prefer_numa=(1,))
    assert len(cpus) == 4 and all(t.cpus[x].numa == 1 for x in cpus)
    assert not set(cpus) & set(p.shared_pool())
    # fractional or burstable -> shared pool
    assert p.allocate({"metadata": {"uid": "u2"}, "status": {"qosClass": "Guaranteed"}},
                      {"name": "c", "resources": {"requests": {"cpu": "1500m"}}}) == p.shared_pool()
    # checkpoint survives a restart
    p2 = StaticPolicy(t, reserved=1, state_file=sf)
    assert p2.assignments == {"u1/c": cpus}
    p2.release_pod("u1")
    assert len(p2.shared_pool()) == 15
    assert json.load(open(sf))["entries"] == {}


def test_cpu_manager_in_kubelet_aligns_with_gpu_numa(run):
    async def main():
        topo = CPUTopology.synthetic(2, 8, 2)
        async with LocalCluster(nodes=1, gpus_per_node=8,
                                kubelet_kwargs={"cpu_manager_policy": "static", "cpu_topology": topo}) as cl:
            c = cl.client
            # GPUs 4-7 are on NUMA 1 in the fixture (numa_per=4): request 8 GPUs... take the second half by
            # first occupying the first four
            pod = {"metadata": {"name": "g", "namespace": "default"},
                   "spec": {"containers": [{"name": "c", "image": "x",
                                            "resources": {"limits": {"cpu": "4", "memory": "1Gi", core.AMD_GPU: "2"},
                                                          "requests": {"cpu": "4", "memory": "1Gi"}}}]}}
            await c.create("pods", pod)
            p = await cl.wait_pod("g")
            assert p["status"]["qosClass"] == "Guaranteed"
            kl = cl.nodes[0].kubelet
            cpus = kl.cpu_manager.assignments[p["metadata"]["uid"] + "/c"]
            numas = set(kl._gpu_numa(p))
            assert len(cpus) == 4 and {topo.cpus[x].numa for x in cpus} <= numas
            await c.delete("pods", "g", "default")
            for _ in range(500):
                if not kl.cpu_manager.assignments:
                    break
                await asyncio.sleep(0.02)
            assert not kl.cpu_manager.assignments
    run(main(), timeout=60)


def test_eviction_thresholds_rank_and_admit():
    th = parse_thresholds("memory.available<100Mi,nodefs.available<10%")
    sig = {"memory.available": (50 << 20, 1 << 30), "nodefs.available": (50, 100)}
    em = EvictionManager(th, lambda: sig, usage_fn=lambda p: int(p["metadata"]["name"][-1]))
    pods = [{"metadata": {"name": "g1"}, "status": {"qosClass": "Guaranteed"}, "spec": {}},
            {"metadata": {"name": "b2"}, "status": {"qosClass": "BestEffort"}, "spec": {"priority": 5}},
            {"metadata": {"name": "b3"}, "status": {"qosClass": "BestEffort"}, "spec": {}}]
    v, msg = em.select_victim(pods)
    assert v["metadata"]["name"] == "b3" and "memory" in msg      # BestEffort, lower priority first
    assert em.has("MemoryPressure") and not em.has("DiskPressure")
    assert em.admit({"status": {"qosClass": "BestEffort"}})[0] == "Evicted"
    assert em.admit({"status": {"qosClass": "Burstable"}}) is None
    sig["memory.available"] = (900 << 20, 1 << 30)
    em.observe()
    assert not em.has("MemoryPressure")


def test_eviction_in_kubelet(run):
    sig = {"memory.available": (8 << 30, 16 << 30)}

    async def main():
        async with LocalCluster(nodes=1, gpus_per_node=0,
                                kubelet_kwargs={"eviction_hard": "memory.available<1Gi", "eviction_signals": lambda: sig,
                                                "eviction_interval": 0.05}) as cl:
            c = cl.client
            for n, res in (("be", {}), ("bu", {"requests": {"memory": "1Gi"}})):
                await c.create("pods", {"metadata": {"name": n, "namespace": "default"},
                                        "spec": {"containers": [{"name": "c", "image": "x", "resources": res}]}})
                await cl.wait_pod(n)
            sig["memory.available"] = (100 << 20, 16 << 30)
            p = await cl.wait_pod("be", phase="Failed", timeout=10)
            assert p["status"]["reason"] == "Evicted"
            for _ in range(300):
                node = await c.get("nodes", "node-0")
                if any(x["type"] == "MemoryPressure" and x["status"] == "True" for x in node["status"]["conditions"]):
                    break
                await asyncio.sleep(0.05)
            else:
                raise AssertionError("MemoryPressure not reported")
            # BestEffort pods: the scheduler keeps them off (CheckNodeMemoryPressure) and the
            # kubelet rejects one bound directly to the node
            await c.create("pods", {"metadata": {"name": "be2", "namespace": "default"},
                                    "spec": {"containers": [{"name": "c", "image": "x"}]}})
            await c.create("pods", {"metadata": {"name": "be3", "namespace": "default"},
                                    "spec": {"nodeName": "node-0", "containers": [{"name": "c", "image": "x"}]}})
            p = await cl.wait_pod("be3", phase="Failed", timeout=10)
            assert p["status"]["reason"] == "Evicted"
            p = await c.get("pods", "be2", "default")
            assert "memory pressure" in p["status"]["conditions"][0]["message"]
    run(main(), timeout=60)


def test_static_pods_mirror(run, tmp_path):
    d = tmp_path / "manifests"
    d.mkdir()
    (d / "web.yaml").write_text("apiVersion: v1\nkind: Pod\nmetadata:\n  name: web\nspec:\n  containers:\n  - name: c\n    image: x\n")

    async def main():
        async with LocalCluster(nodes=1, gpus_per_node=0, kubelet_kwargs={"pod_manifest_path": str(d)}) as cl:
            kl = cl.nodes[0].kubelet
            kl.static_pods.period = 0.1
            p = await cl.wait_pod("web-node-0", timeout=10)
            assert p["metadata"]["annotations"]["kubernetes.io/config.source"] == "file"
            assert p["spec"]["nodeName"] == "node-0"
            # deleting the mirror pod re-creates it
            uid = p["metadata"]["uid"]
            await cl.client.delete("pods", "web-node-0", "default", grace_period=0)

            async def recreated():
                try:
                    q = await cl.client.get("pods", "web-node-0", "default")
                    return q["metadata"]["uid"] != uid and q["status"].get("phase") == "Running"
                except Exception:
                    return False
            for _ in range(200):
                if await recreated():
                    break
                await asyncio.sleep(0.05)
            assert await recreated()
            # removing the manifest deletes the mirror pod
            os.remove(d / "web.yaml")
            for _ in range(200):
                try:
                    await cl.client.get("pods", "web-node-0", "default")
                except Exception:
                    break
                await asyncio.sleep(0.05)
            else:
                raise AssertionError("mirror pod not deleted")
    run(main(), timeout=60)


# -- cpu_assignment_test.go TestTakeByTopology --------------------------------------------------

def _topo(details):
    from kubernetes_amd.kubelet.cpumanager import CPUInfo, CPUTopology
    return CPUTopology([CPUInfo(cpu, core, sock, sock) for cpu, (core, sock) in details.items()])


SINGLE_SOCKET_HT = {0: (0, 0), 1: (1, 0), 2: (2, 0), 3: (3, 0), 4: (0, 0), 5: (1, 0), 6: (2, 0), 7: (3, 0)}
DUAL_SOCKET_HT = {0: (0, 0), 1: (1, 1), 2: (2, 0), 3: (3, 1), 4: (4, 0), 5: (5, 1),
                  6: (0, 0), 7: (1, 1), 8: (2, 0), 9: (3, 1), 10: (4, 0), 11: (5, 1)}
DUAL_SOCKET_NO_HT = {0: (0, 0), 1: (1, 0), 2: (2, 0), 3: (3, 0), 4: (4, 1), 5: (5, 1), 6: (6, 1), 7: (7, 1)}


@pytest.mark.parametrize("topo,avail,n,want", [
    (SINGLE_SOCKET_HT, {0, 2, 4, 6}, 5, None),
    (SINGLE_SOCKET_HT, set(range(8)), 0, []),
    (SINGLE_SOCKET_HT, set(range(8)), 1, [0]),
    (SINGLE_SOCKET_HT, {1, 3, 5, 6, 7}, 1, [6]),
    (SINGLE_SOCKET_HT, set(range(8)), 2, [0, 4]),
    (SINGLE_SOCKET_HT, set(range(8)), 8, list(range(8))),
    (SINGLE_SOCKET_HT, {0, 1, 2, 3, 6}, 2, [2, 6]),
    (DUAL_SOCKET_HT, {1, 2, 3, 4, 5, 7, 8, 9, 10, 11}, 1, [2]),
    (DUAL_SOCKET_HT, set(range(12)), 6, [0, 2, 4, 6, 8, 10]),
    (DUAL_SOCKET_NO_HT, set(range(8)), 4, [0, 1, 2, 3]),
    (DUAL_SOCKET_NO_HT, {1, 2, 3, 4, 5, 6, 7}, 1, [1]),
], ids=["more than available", "zero", "one", "one, some taken", "two", "all", "two, one free core",
        "dual socket one cpu", "dual socket a socket", "no HT a socket", "no HT one"])
def test_take_by_topology(topo, avail, n, want):
    from kubernetes_amd.kubelet.cpumanager import take_by_topology
    if want is None:
        with pytest.raises(ValueError, match="not enough cpus available to satisfy request"):
            take_by_topology(_topo(topo), avail, n)
    else:
        assert take_by_topology(_topo(topo), avail, n) == want


# -- policy_static_test.go TestStaticPolicyAdd (allocation from the default set minus reserved) --

@pytest.mark.parametrize("topo,default,req,lim,want", [
    (SINGLE_SOCKET_HT, set(range(8)), "8000m", "8000m", "error"),
    (SINGLE_SOCKET_HT, set(range(8)), "1000m", "1000m", [4]),          # sibling of the partial core
    (SINGLE_SOCKET_HT, {0, 1, 4, 5}, "2000m", "2000m", [1, 5]),
    (DUAL_SOCKET_HT, {0, 1, 3, 4, 5, 6, 7, 8, 9, 10, 11}, "6000m", "6000m", [1, 3, 5, 7, 9, 11]),
    (DUAL_SOCKET_HT, {0, 2, 3, 4, 6, 7, 8, 9, 10, 11}, "6000m", "6000m", [2, 3, 4, 8, 9, 10]),
    (DUAL_SOCKET_NO_HT, {0, 1, 3, 4, 5, 6, 7}, "4000m", "4000m", [4, 5, 6, 7]),
    (DUAL_SOCKET_NO_HT, {0, 1, 3, 6, 7}, "4000m", "4000m", [1, 3, 6, 7]),
    (DUAL_SOCKET_HT, {0, 1, 3, 4, 5, 6, 7, 8, 9, 10, 11}, "8000m", "8000m", [1, 3, 4, 5, 7, 9, 10, 11]),
    (SINGLE_SOCKET_HT, set(range(8)), "1000m", "2000m", None),           # not Guaranteed
    (SINGLE_SOCKET_HT, set(range(8)), "977m", "977m", None),             # non-integer CPUs
    (SINGLE_SOCKET_HT, {0, 7}, "2000m", "2000m", "error"),
    (DUAL_SOCKET_HT, {0, 4, 5, 6, 7, 8, 9, 10, 11}, "10000m", "10000m", "error"),
], ids=["SingleCore expect error", "alloc one cpu", "alloc one core", "dual HT one socket", "dual HT three cores",
        "no HT one socket", "no HT four cores", "dual HT socket + core", "non-Gu pod", "non-integer", "no alloc error",
        "dual HT error"])
def test_static_policy_add(topo, default, req, lim, want):
    t = _topo(topo)
    pod = {"metadata": {"uid": "u"}, "spec": {"containers": [{"name": "c", "resources": {
        "requests": {"cpu": req, "memory": "1G"}, "limits": {"cpu": lim, "memory": "1G"}}}]},
        "status": {"qosClass": "Guaranteed" if req == lim else "Burstable"}}
    n = StaticPolicy.guaranteed_cpus(pod, pod["spec"]["containers"][0])
    if want is None:
        assert n == 0
        return
    reserved = set(take_by_topology(t, set(t.cpus), 1))      # NewStaticPolicy(topo, 1): cpu 0
    assert reserved == {0}
    if want == "error":
        with pytest.raises(ValueError, match="not enough cpus available to satisfy request"):
            take_by_topology(t, default - reserved, n)
    else:
        assert take_by_topology(t, default - reserved, n) == want


# -- kubelet_pods_test.go TestPodPhaseWithRestart{Always,Never,OnFailure} ------------------------

def _running(n):
    return {"name": n, "state": {"running": {}}}


def _stopped(n, code=0):
    return {"name": n, "state": {"terminated": {"exitCode": code}}}


def _waiting(n):
    return {"name": n, "state": {"waiting": {}}}


def _waiting_last(n):
    return {"name": n, "state": {"waiting": {}}, "lastState": {"terminated": {"exitCode": 0}}}


PHASE_CASES = {
    "Always": [([], "Pending"), ([_running("A"), _running("B")], "Running"),
               ([_stopped("A"), _stopped("B")], "Running"), ([_running("A"), _stopped("B")], "Running"),
               ([_running("A")], "Pending"), ([_running("A"), _waiting("B")], "Pending"),
               ([_running("A"), _waiting_last("B")], "Running")],
    "Never": [([], "Pending"), ([_running("A"), _running("B")], "Running"),
              ([_stopped("A"), _stopped("B")], "Succeeded"), ([_stopped("A", -1), _stopped("B", -1)], "Failed"),
              ([_running("A"), _stopped("B")], "Running"), ([_running("A")], "Pending"),
              ([_running("A"), _waiting("B")], "Pending")],
    "OnFailure": [([], "Pending"), ([_running("A"), _running("B")], "Running"),
                  ([_stopped("A"), _stopped("B")], "Succeeded"), ([_stopped("A", -1), _stopped("B", -1)], "Running"),
                  ([_running("A"), _stopped("B")], "Running"), ([_running("A")], "Pending"),
                  ([_running("A"), _waiting("B")], "Pending"), ([_running("A"), _waiting_last("B")], "Running")],
}


@pytest.mark.parametrize("policy,statuses,want", [(p, s, w) for p, cases in PHASE_CASES.items() for s, w in cases])
def test_pod_phase(policy, statuses, want):
    from kubernetes_amd.kubelet.kubelet import get_phase
    spec = {"containers": [{"name": "A"}, {"name": "B"}], "restartPolicy": policy}
    assert get_phase(spec, statuses) == want


@pytest.mark.parametrize("policy,init,want", [
    ("Never", [_stopped("i", 1)], "Failed"), ("Always", [_stopped("i", 1)], "Pending"),
    ("Always", [_running("i")], "Pending"), ("Always", [_stopped("i")], "Running"),
    ("OnFailure", [{"name": "i", "state": {"waiting": {}}, "lastState": {"terminated": {"exitCode": 2}}}], "Pending"),
])
def test_pod_phase_with_init_containers(policy, init, want):
    """GetPhase's init-container accounting (kubelet_pods.go: pendingInitialization /
    failedInitialization); the regular containers run once initialization is done."""
    from kubernetes_amd.kubelet.kubelet import get_phase
    spec = {"initContainers": [{"name": "i"}], "containers": [{"name": "A"}], "restartPolicy": policy}
    statuses = [_running("A")] if want == "Running" else []
    assert get_phase(spec, statuses, init) == want


# -- pkg/kubelet/cm/cpuset/cpuset_test.go TestCPUSetString / TestParse ---------------------------
@pytest.mark.parametrize("cpus,text", [((), ""), ((5,), "5"), ((1, 2, 3, 4, 5), "1-5"), ((1, 2, 3, 5, 6, 8), "1-3,5-6,8")])
def test_cpuset_string(cpus, text):
    from kubernetes_amd.kubelet.cpumanager import format_cpulist
    assert format_cpulist(cpus) == text


@pytest.mark.parametrize("text,cpus", [("", set()), ("5", {5}), ("1,2,3,4,5", {1, 2, 3, 4, 5}), ("1-5", {1, 2, 3, 4, 5}),
                                       ("1-2,3-5", {1, 2, 3, 4, 5})])
def test_cpuset_parse(text, cpus):
    from kubernetes_amd.kubelet.cpumanager import parse_cpulist
    assert set(parse_cpulist(text)) == cpus


def test_static_pod_defaults_like_apply_defaults():
    """`pkg/kubelet/config/common.go` applyDefaults: `<name>-<lower-cased node>`, namespace
    default for an empty one, bound to the node, and file pods tolerate every NoExecute taint
    (added once); pods from a URL do not get the toleration."""
    from types import SimpleNamespace

    from kubernetes_amd.kubelet.config import CONFIG_HASH, CONFIG_SOURCE, StaticPodSource
    src = StaticPodSource(SimpleNamespace(node_name="Node-A"), None)
    doc = {"metadata": {"name": "etcd", "namespace": ""}, "spec": {"containers": [{"name": "c", "image": "i"}],
                                                                   "tolerations": [{"key": "k", "operator": "Exists"}]}}
    pod = src._mirror(doc, "h1", "file")
    assert pod["metadata"]["name"] == "etcd-node-a" and pod["metadata"]["namespace"] == "default"
    assert pod["spec"]["nodeName"] == "Node-A"
    assert pod["metadata"]["annotations"][CONFIG_SOURCE] == "file" and pod["metadata"]["annotations"][CONFIG_HASH] == "h1"
    assert pod["spec"]["tolerations"] == [{"key": "k", "operator": "Exists"}, {"operator": "Exists", "effect": "NoExecute"}]
    again = src._mirror(pod, "h1", "file")
    assert again["spec"]["tolerations"].count({"operator": "Exists", "effect": "NoExecute"}) == 1
    assert "tolerations" not in src._mirror({"metadata": {"name": "x"}, "spec": {}}, "h2", "http")["spec"]
