"""Scheduler cache — port of `plugin/pkg/scheduler/schedulercache/cache_test.go`
(TestAssumePodScheduled, TestExpirePod, TestAddPodWillConfirm, TestAddPodWillReplaceAssumed,
TestAddPodAfterExpiration, TestUpdatePod, TestExpireAddUpdatePod, TestRemovePod, TestForgetPod)
plus the fork's device accounting through assume / forget / expiry."""
import time

from kubernetes_amd.scheduler.cache import DEFAULT_MEMORY, DEFAULT_MILLI_CPU, SchedulerCache

from test_scheduler import gpu_dev, gpu_pod, node as gpu_node


def base_pod(node, name, cpu, mem, extended="", ports=()):
    req = {}
    if cpu:
        req["cpu"] = cpu
    if mem:
        req["memory"] = mem
    if extended:
        k, v = extended.rsplit(":", 1)
        req[k] = v
    return {"metadata": {"name": name, "namespace": "node_info_cache_test", "uid": f"uid-{name}"},
            "spec": {"nodeName": node, "containers": [{"name": "c", "resources": {"requests": req},
                                                      "ports": [dict(p) for p in ports]}]}}


P80 = [{"hostIP": "127.0.0.1", "hostPort": 80, "protocol": "TCP"}]
P8080 = [{"hostIP": "127.0.0.1", "hostPort": 8080, "protocol": "TCP"}]


def state(ni):
    if ni is None:
        return None
    return {"cpu": ni.req_cpu, "mem": ni.req_mem, "nz": (ni.nz_cpu, ni.nz_mem), "scalars": {k: v for k, v in ni.req_scalars.items() if v},
            "pods": sorted(p["metadata"]["name"] for p, _ in ni.pods.values()),
            "ports": sorted(f"{proto}/{ip}/{port}" for ip, proto, port in ni.ports)}


def test_assume_pod_scheduled():
    pods = [base_pod("node", "test", "100m", "500", ports=P80), base_pod("node", "test-1", "100m", "500", ports=P80),
            base_pod("node", "test-2", "200m", "1Ki", ports=P8080), base_pod("node", "test-nonzero", "", "", ports=P80),
            base_pod("node", "test", "100m", "500", "example.com/foo:3", P80),
            base_pod("node", "test-2", "200m", "1Ki", "example.com/foo:5", P8080),
            base_pod("node", "test", "100m", "500", "random-invalid-extended-key:100", [{}])]
    cases = [
        ([0], {"cpu": 100, "mem": 500, "nz": (100, 500), "scalars": {}, "pods": ["test"], "ports": ["TCP/127.0.0.1/80"]}),
        ([1, 2], {"cpu": 300, "mem": 1524, "nz": (300, 1524), "scalars": {}, "pods": ["test-1", "test-2"],
                  "ports": ["TCP/127.0.0.1/80", "TCP/127.0.0.1/8080"]}),
        ([3], {"cpu": 0, "mem": 0, "nz": (DEFAULT_MILLI_CPU, DEFAULT_MEMORY), "scalars": {}, "pods": ["test-nonzero"],
               "ports": ["TCP/127.0.0.1/80"]}),
        ([4], {"cpu": 100, "mem": 500, "nz": (100, 500), "scalars": {"example.com/foo": 3}, "pods": ["test"],
               "ports": ["TCP/127.0.0.1/80"]}),
        ([4, 5], {"cpu": 300, "mem": 1524, "nz": (300, 1524), "scalars": {"example.com/foo": 8}, "pods": ["test", "test-2"],
                  "ports": ["TCP/127.0.0.1/80", "TCP/127.0.0.1/8080"]}),
        ([6], {"cpu": 100, "mem": 500, "nz": (100, 500), "scalars": {}, "pods": ["test"], "ports": []}),
    ]
    for idx, want in cases:
        c = SchedulerCache(assumed_ttl=1)
        for i in idx:
            c.assume_pod(pods[i])
        assert state(c.nodes["node"]) == want, idx
        for i in idx:
            c.forget_pod(pods[i])
        assert "node" not in c.nodes                     # NodeInfo cleaned up


def test_expire_pod():
    p1, p2 = base_pod("node", "test-1", "100m", "500", ports=P80), base_pod("node", "test-2", "200m", "1Ki", ports=P8080)
    now = time.monotonic()
    c = SchedulerCache(assumed_ttl=10)
    c.assume_pod(p1)
    c.finish_binding(p1)
    c.cleanup_expired(now + 20 + 1)
    assert "node" not in c.nodes
    c = SchedulerCache(assumed_ttl=10)
    c.assume_pod(p1)
    c.finish_binding(p1)
    c.assume_pod(p2)
    c.finish_binding(p2)
    c.assumed[f"node_info_cache_test/test-2"] = now + 15 + 10       # assumed 15 s later
    c.cleanup_expired(now + 20 + 1)
    assert state(c.nodes["node"])["pods"] == ["test-2"] and c.nodes["node"].req_cpu == 200


def test_add_pod_will_confirm_and_replace_assumed():
    p1, p2 = base_pod("node", "test-1", "100m", "500", ports=P80), base_pod("node", "test-2", "200m", "1Ki", ports=P8080)
    c = SchedulerCache(assumed_ttl=10)
    for p in (p1, p2):
        c.assume_pod(p)
        c.finish_binding(p)
    c.add_pod(p1)                                        # confirmed: survives expiry
    c.cleanup_expired(time.monotonic() + 21)
    assert state(c.nodes["node"])["pods"] == ["test-1"]
    # an Add on another node replaces the assumed pod; an Update then changes it
    assumed = base_pod("assumed-node", "test-1", "100m", "500", ports=[{"hostPort": 80}])
    added = base_pod("actual-node", "test-1", "100m", "500", ports=[{"hostPort": 80}])
    updated = base_pod("actual-node", "test-1", "200m", "500", ports=[{"hostPort": 90}])
    c = SchedulerCache(assumed_ttl=10)
    c.assume_pod(assumed)
    c.finish_binding(assumed)
    c.add_pod(added)
    c.update_pod(added, updated)
    assert "assumed-node" not in c.nodes
    assert state(c.nodes["actual-node"]) == {"cpu": 200, "mem": 500, "nz": (200, 500), "scalars": {}, "pods": ["test-1"],
                                             "ports": ["TCP/0.0.0.0/90"]}


def test_add_after_expiration_update_and_remove():
    p = base_pod("node", "test", "100m", "500", ports=P80)
    q = base_pod("node", "test", "200m", "1Ki", ports=P8080)
    c = SchedulerCache(assumed_ttl=10)
    c.assume_pod(p)
    c.finish_binding(p)
    c.cleanup_expired(time.monotonic() + 21)
    assert "node" not in c.nodes
    c.add_pod(p)
    assert state(c.nodes["node"])["cpu"] == 100
    for old, new, cpu, ports in ((p, q, 200, ["TCP/127.0.0.1/8080"]), (q, p, 100, ["TCP/127.0.0.1/80"])):
        c.update_pod(old, new)
        assert state(c.nodes["node"])["cpu"] == cpu and state(c.nodes["node"])["ports"] == ports
    c.remove_pod(p)
    assert "node" not in c.nodes


def test_device_accounting_follows_assume_forget_and_expiry():
    """Fork F5: assumed pods hold their devices (the assume carries `assigned`); forgetting or
    expiring the assumption frees them, a confirmed pod keeps them."""
    c = SchedulerCache(assumed_ttl=10)
    c.add_node(gpu_node("n0", [gpu_dev(i) for i in range(4)]))
    p = gpu_pod("p", 2)
    p["spec"]["nodeName"] = "n0"
    p["spec"]["extendedResources"][0]["assigned"] = ["g0", "g1"]
    c.assume_pod(p)
    er = c.nodes["n0"].er
    assert er.free_count("amd.com/gpu") == 2 and set(er.used["amd.com/gpu"]) == {"g0", "g1"}
    c.forget_pod(p)
    assert er.free_count("amd.com/gpu") == 4 and not er.used
    c.assume_pod(p)
    c.finish_binding(p)
    c.cleanup_expired(time.monotonic() + 11)
    assert er.free_count("amd.com/gpu") == 4
    c.assume_pod(p)
    c.finish_binding(p)
    c.add_pod(p)                                         # confirmed by the informer
    c.cleanup_expired(time.monotonic() + 11)
    assert er.free_count("amd.com/gpu") == 2
