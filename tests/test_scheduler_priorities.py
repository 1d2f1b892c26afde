"""Scheduler priority functions against the reference's own tables
(`plugin/pkg/scheduler/algorithm/priorities/{least_requested,most_requested,
balanced_resource_allocation,selector_spreading,taint_toleration,node_affinity}_test.go`):
integer scores as the reference computes them (non-zero default requests per container,
NormalizeReduce, the zone-weighted spread reduce)."""
import itertools

import pytest

from kubernetes_amd.scheduler.cache import PodInfo, SchedulerCache
from kubernetes_amd.scheduler.generic import CycleContext, GenericScheduler

_uid = itertools.count()


def node(name, cpu_milli=4000, mem=10000, labels=None, taints=None):
    return {"metadata": {"name": name, "labels": dict(labels or {})}, "spec": {"taints": list(taints or [])},
            "status": {"allocatable": {"cpu": f"{cpu_milli}m", "memory": str(mem), "pods": "110"},
                       "conditions": [{"type": "Ready", "status": "True"}]}}


def pod(node_name="", containers=(), labels=None, ns="default", spec=None, owner=None):
    n = next(_uid)
    p = {"metadata": {"name": f"p{n}", "namespace": ns, "uid": f"u{n}", "labels": dict(labels or {})},
         "spec": dict(spec or {}, containers=[{"name": f"c{i}", "resources": {"requests": r}} if r is not None
                                              else {"name": f"c{i}"} for i, r in enumerate(containers)])}
    if node_name:
        p["spec"]["nodeName"] = node_name
    if owner:
        p["metadata"]["ownerReferences"] = [{"uid": owner, "controller": True, "kind": "ReplicaSet", "name": "rs"}]
    return p


def scores(priority, the_pod, nodes, pods=(), services=()):
    cache = SchedulerCache()
    for n in nodes:
        cache.add_node(n)
    for p in pods:
        cache.add_pod(p)
    for s in services:
        cache.set_service(s)
    gs = GenericScheduler(cache, priorities={priority: 1})
    nis = [cache.nodes[n["metadata"]["name"]] for n in nodes]
    ctx = CycleContext(cache, the_pod)
    prios = [e for e in gs.priorities]           # every configured priority, even all-equal ones
    raws = [tuple(fn(the_pod, PodInfo(the_pod), ni, ctx) for _, _, fn, _, _ in prios) for ni in nis]
    got = gs._combine(prios, nis, raws)
    return [int(got[n["metadata"]["name"]]) for n in nodes]


CPU_ONLY = [{"cpu": "1000m", "memory": "0"}, {"cpu": "2000m", "memory": "0"}]
CPU_AND_MEM = [{"cpu": "1000m", "memory": "2000"}, {"cpu": "2000m", "memory": "3000"}]


@pytest.mark.parametrize("the_pod,nodes,pods,expect", [
    (pod(), [node("machine1", 4000, 10000), node("machine2", 4000, 10000)], [], [10, 10]),
    (pod(containers=CPU_AND_MEM), [node("machine1", 4000, 10000), node("machine2", 6000, 10000)], [], [3, 5]),
    (pod(), [node("machine1", 4000, 10000), node("machine2", 4000, 10000)],
     [pod("machine1"), pod("machine1"), pod("machine2"), pod("machine2")], [10, 10]),
    (pod(), [node("machine1", 10000, 20000), node("machine2", 10000, 20000)],
     [pod("machine1", CPU_ONLY), pod("machine1", CPU_ONLY), pod("machine2", CPU_ONLY), pod("machine2", CPU_AND_MEM)], [7, 5]),
    (pod(containers=CPU_AND_MEM), [node("machine1", 10000, 20000), node("machine2", 10000, 20000)],
     [pod("machine1", CPU_ONLY), pod("machine2", CPU_AND_MEM)], [5, 4]),
    (pod(containers=CPU_AND_MEM), [node("machine1", 10000, 20000), node("machine2", 10000, 50000)],
     [pod("machine1", CPU_ONLY), pod("machine2", CPU_AND_MEM)], [5, 6]),
    (pod(containers=CPU_ONLY), [node("machine1", 4000, 10000), node("machine2", 4000, 10000)],
     [pod("machine1", CPU_ONLY), pod("machine2", CPU_AND_MEM)], [5, 2]),
    (pod(), [node("machine1", 0, 0), node("machine2", 0, 0)],
     [pod("machine1", CPU_ONLY), pod("machine2", CPU_AND_MEM)], [0, 0]),
])
def test_least_requested(the_pod, nodes, pods, expect):
    assert scores("LeastRequestedPriority", the_pod, nodes, pods) == expect


BIG_CPU_AND_MEM = [{"cpu": "2000m", "memory": "4000"}, {"cpu": "3000m", "memory": "5000"}]


@pytest.mark.parametrize("the_pod,nodes,pods,expect", [
    (pod(), [node("machine1", 4000, 10000), node("machine2", 4000, 10000)], [], [0, 0]),
    (pod(containers=CPU_AND_MEM), [node("machine1", 4000, 10000), node("machine2", 6000, 10000)], [], [6, 5]),
    (pod(), [node("machine1", 10000, 20000), node("machine2", 10000, 20000)],
     [pod("machine1", CPU_ONLY), pod("machine1", CPU_ONLY), pod("machine2", CPU_ONLY), pod("machine2", CPU_AND_MEM)], [3, 4]),
    (pod(containers=CPU_AND_MEM), [node("machine1", 10000, 20000), node("machine2", 10000, 20000)],
     [pod("machine1", CPU_ONLY), pod("machine2", CPU_AND_MEM)], [4, 5]),
    (pod(containers=BIG_CPU_AND_MEM), [node("machine1", 4000, 10000), node("machine2", 10000, 8000)], [], [4, 2]),
])
def test_most_requested(the_pod, nodes, pods, expect):
    assert scores("MostRequestedPriority", the_pod, nodes, pods) == expect


@pytest.mark.parametrize("the_pod,nodes,pods,expect", [
    (pod(), [node("machine1", 4000, 10000), node("machine2", 4000, 10000)], [], [10, 10]),
    (pod(containers=CPU_AND_MEM), [node("machine1", 4000, 10000), node("machine2", 6000, 10000)], [], [7, 10]),
    (pod(), [node("machine1", 4000, 10000), node("machine2", 4000, 10000)],
     [pod("machine1"), pod("machine1"), pod("machine2"), pod("machine2")], [10, 10]),
    (pod(), [node("machine1", 10000, 20000), node("machine2", 10000, 20000)],
     [pod("machine1", CPU_ONLY), pod("machine1", CPU_ONLY), pod("machine2", CPU_ONLY), pod("machine2", CPU_AND_MEM)], [4, 6]),
    (pod(containers=CPU_AND_MEM), [node("machine1", 10000, 20000), node("machine2", 10000, 20000)],
     [pod("machine1", CPU_ONLY), pod("machine2", CPU_AND_MEM)], [6, 9]),
    (pod(containers=CPU_AND_MEM), [node("machine1", 10000, 20000), node("machine2", 10000, 50000)],
     [pod("machine1", CPU_ONLY), pod("machine2", CPU_AND_MEM)], [6, 6]),
    (pod(containers=CPU_ONLY), [node("machine1", 4000, 10000), node("machine2", 4000, 10000)],
     [pod("machine1", CPU_ONLY), pod("machine2", CPU_AND_MEM)], [0, 0]),
])
def test_balanced_resource_allocation(the_pod, nodes, pods, expect):
    assert scores("BalancedResourceAllocation", the_pod, nodes, pods) == expect


ZONE = "failure-domain.beta.kubernetes.io/zone"
Z = ["machine1.zone1", "machine1.zone2", "machine2.zone2", "machine1.zone3", "machine2.zone3", "machine3.zone3"]
L1 = {"label1": "l1", "baz": "blah"}
L2 = {"label2": "l2", "baz": "blah"}


def zone_nodes():
    return [node(n, labels={ZONE: n.split(".")[1]}) for n in Z]


def svc(selector):
    return {"metadata": {"name": "s", "namespace": "default"}, "spec": {"selector": selector}}


@pytest.mark.parametrize("placed,expect", [
    ([("machine1.zone1", L2), ("machine1.zone2", L1)], [10, 0, 3, 10, 10, 10]),
    ([("machine1.zone1", L2), ("machine1.zone2", L1), ("machine2.zone2", L1), ("machine1.zone3", L2),
      ("machine2.zone3", L1)], [10, 0, 0, 6, 3, 6]),
    ([("machine1.zone1", L2), ("machine1.zone2", L2)], [10] * 6),
])
def test_zone_selector_spread(placed, expect):
    """TestZoneSelectorSpreadPriority: node count blended 1/3 : 2/3 with the zone count."""
    pods = [pod(n, labels=lbl) for n, lbl in placed]
    assert scores("SelectorSpreadPriority", pod(labels=L1), zone_nodes(), pods, [svc(L1)]) == expect


def test_selector_spread_without_zones_and_deleted_pods():
    """TestSelectorSpreadPriority "three pods, two service pods on different machines": a
    deleted predecessor is ignored."""
    nodes = [node("machine1"), node("machine2")]
    pods = [pod("machine1", labels=L2), pod("machine1", labels=L1), pod("machine2", labels=L1), pod("machine2", labels=L1)]
    assert scores("SelectorSpreadPriority", pod(labels=L1), nodes, pods, [svc(L1)]) == [5, 0]
    pods[3]["metadata"]["deletionTimestamp"] = "2000-01-01T00:00:00Z"
    assert scores("SelectorSpreadPriority", pod(labels=L1), nodes, pods, [svc(L1)]) == [0, 0]


def test_taint_toleration_priority():
    """TestTaintAndToleration: fewer intolerable PreferNoSchedule taints score higher."""
    taints = [{"key": "foo", "value": "bar", "effect": "PreferNoSchedule"},
              {"key": "cpu-type", "value": "arm64", "effect": "PreferNoSchedule"}]
    nodes = [node("nodeA", taints=taints), node("nodeB", taints=taints[:1]), node("nodeC")]
    p = pod(spec={"tolerations": [{"key": "cpu-type", "operator": "Equal", "value": "arm64",
                                   "effect": "PreferNoSchedule"}]})
    assert scores("TaintTolerationPriority", p, nodes) == [0, 0, 10]
    assert scores("TaintTolerationPriority", pod(), nodes) == [0, 5, 10]


def test_node_affinity_priority():
    """TestNodeAffinityPriority "all machines matches the preferred scheduling requirements"."""
    aff = {"nodeAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": [
        {"weight": 2, "preference": {"matchExpressions": [{"key": "foo", "operator": "In", "values": ["bar"]}]}},
        {"weight": 4, "preference": {"matchExpressions": [{"key": "key", "operator": "In", "values": ["value"]}]}},
        {"weight": 5, "preference": {"matchExpressions": [
            {"key": "foo", "operator": "In", "values": ["bar"]}, {"key": "key", "operator": "In", "values": ["value"]},
            {"key": "az", "operator": "In", "values": ["az1"]}]}}]}}
    nodes = [node("machine1", labels={"foo": "bar"}), node("machine5", labels={"foo": "bar", "key": "value", "az": "az1"}),
             node("machine2", labels={"key": "value"})]
    assert scores("NodeAffinityPriority", pod(spec={"affinity": aff}), nodes) == [1, 10, 3]
