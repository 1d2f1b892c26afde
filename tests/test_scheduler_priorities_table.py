"""Ported resource-priority tables.

Reference: `plugin/pkg/scheduler/algorithm/priorities/least_requested_test.go`,
`most_requested_test.go` and `balanced_resource_allocation_test.go`: the same fixtures
(`cpuOnly`, `cpuAndMemory`, `bigCpuAndMemory`, pods with no containers) and the expected
per-node integer scores. A container request set explicitly to 0 counts as 0; only a missing
request takes the non-zero default (priorities/util/non_zero.go).
"""
import pytest

from kubernetes_amd.scheduler.cache import PodInfo, SchedulerCache
from kubernetes_amd.scheduler.generic import CycleContext, GenericScheduler


def _ctr(cpu, mem):
    return {"name": "c", "resources": {"requests": {"cpu": cpu, "memory": mem}}}


CPU_ONLY = [_ctr("1000m", "0"), _ctr("2000m", "0")]
CPU_AND_MEM = [_ctr("1000m", "2000"), _ctr("2000m", "3000")]
BIG = [_ctr("2000m", "4000"), _ctr("3000m", "5000")]
NONE = []


def _pod(containers, node=None, i=0):
    spec = {"containers": containers}
    if node:
        spec["nodeName"] = node
    return {"metadata": {"name": f"p{i}", "namespace": "default", "uid": f"u{i}"}, "spec": spec,
            "status": {"phase": "Running"}}


def _node(name, cpu_m, mem):
    alloc = {"cpu": f"{cpu_m}m", "memory": str(mem), "pods": "100"}
    return {"metadata": {"name": name}, "spec": {},
            "status": {"allocatable": alloc, "capacity": dict(alloc), "conditions": [{"type": "Ready", "status": "True"}]}}


M1 = ("machine1", "machine1")

# (name, pod containers, nodes [(cpu_m, mem)], existing pods [(containers, node)], {priority: [s1, s2]})
CASES = [
    ("nothing scheduled, nothing requested", NONE, [(4000, 10000), (4000, 10000)], [],
     {"LeastRequestedPriority": [10, 10], "MostRequestedPriority": [0, 0], "BalancedResourceAllocation": [10, 10]}),
    ("nothing scheduled, resources requested, differently sized machines", CPU_AND_MEM,
     [(4000, 10000), (6000, 10000)], [],
     {"LeastRequestedPriority": [3, 5], "MostRequestedPriority": [6, 5], "BalancedResourceAllocation": [7, 10]}),
    ("no resources requested, pods scheduled", NONE, [(4000, 10000), (4000, 10000)],
     [(NONE, "machine1"), (NONE, "machine1"), (NONE, "machine2"), (NONE, "machine2")],
     {"LeastRequestedPriority": [10, 10], "BalancedResourceAllocation": [10, 10]}),
    ("no resources requested, pods scheduled with resources", NONE, [(10000, 20000), (10000, 20000)],
     [(CPU_ONLY, "machine1"), (CPU_ONLY, "machine1"), (CPU_ONLY, "machine2"), (CPU_AND_MEM, "machine2")],
     {"LeastRequestedPriority": [7, 5], "MostRequestedPriority": [3, 4], "BalancedResourceAllocation": [4, 6]}),
    ("resources requested, pods scheduled with resources", CPU_AND_MEM, [(10000, 20000), (10000, 20000)],
     [(CPU_ONLY, "machine1"), (CPU_AND_MEM, "machine2")],
     {"LeastRequestedPriority": [5, 4], "MostRequestedPriority": [4, 5], "BalancedResourceAllocation": [6, 9]}),
    ("resources requested, pods scheduled with resources, differently sized machines", CPU_AND_MEM,
     [(10000, 20000), (10000, 50000)], [(CPU_ONLY, "machine1"), (CPU_AND_MEM, "machine2")],
     {"LeastRequestedPriority": [5, 6], "BalancedResourceAllocation": [6, 6]}),
    ("requested resources exceed node capacity", CPU_ONLY, [(4000, 10000), (4000, 10000)],
     [(CPU_ONLY, "machine1"), (CPU_AND_MEM, "machine2")],
     {"LeastRequestedPriority": [5, 2], "BalancedResourceAllocation": [0, 0]}),
    ("zero node resources, pods scheduled with resources", NONE, [(0, 0), (0, 0)],
     [(CPU_ONLY, "machine1"), (CPU_AND_MEM, "machine2")],
     {"LeastRequestedPriority": [0, 0], "BalancedResourceAllocation": [0, 0]}),
    ("resources requested with more than the node", BIG, [(4000, 10000), (10000, 8000)], [],
     {"MostRequestedPriority": [4, 2]}),
]


@pytest.mark.parametrize("name,ctrs,nodes,pods,expected", CASES, ids=[c[0] for c in CASES])
def test_resource_priorities(name, ctrs, nodes, pods, expected):
    cache = SchedulerCache()
    for i, (cpu, mem) in enumerate(nodes):
        cache.add_node(_node(f"machine{i + 1}", cpu, mem))
    for i, (c, n) in enumerate(pods):
        cache.add_pod(_pod(c, n, i + 1))
    pod = _pod(ctrs)
    infos = [cache.nodes["machine1"], cache.nodes["machine2"]]
    for prio, want in expected.items():
        gs = GenericScheduler(cache, [], {prio: 1}, equivalence_cache=False)
        scores = gs.prioritize(pod, PodInfo(pod), infos, CycleContext(cache, pod))
        assert [scores["machine1"], scores["machine2"]] == want, (name, prio)


# -- image_locality_test.go ----------------------------------------------------------------------

MB = 1024 * 1024
NODE_40_140_2000 = [(["gcr.io/40", "gcr.io/40:v1"], 40 * MB), (["gcr.io/140", "gcr.io/140:v1"], 140 * MB),
                    (["gcr.io/2000"], 2000 * MB)]
NODE_250_10 = [(["gcr.io/250"], 250 * MB), (["gcr.io/10", "gcr.io/10:v1"], 10 * MB)]


@pytest.mark.parametrize("images,want", [
    (["gcr.io/40", "gcr.io/250"], [1, 3]),          # two images spread on two nodes, prefer the larger one
    (["gcr.io/40", "gcr.io/140"], [2, 0]),          # two images on one node, prefer this node
    (["gcr.io/10", "gcr.io/2000"], [10, 0]),        # if exceed limit, use limit
])
def test_image_locality(images, want):
    cache = SchedulerCache()
    for name, imgs in (("machine1", NODE_40_140_2000), ("machine2", NODE_250_10)):
        n = _node(name, 4000, 10000)
        n["status"]["images"] = [{"names": names, "sizeBytes": size} for names, size in imgs]
        cache.add_node(n)
    pod = _pod([{"name": f"c{i}", "image": im} for i, im in enumerate(images)])
    gs = GenericScheduler(cache, [], {"ImageLocalityPriority": 1}, equivalence_cache=False)
    scores = gs.prioritize(pod, PodInfo(pod), [cache.nodes["machine1"], cache.nodes["machine2"]],
                           CycleContext(cache, pod))
    assert [scores["machine1"], scores["machine2"]] == want


# -- node_prefer_avoid_pods_test.go --------------------------------------------------------------

def _avoid(kind, uid):
    import json
    return {"scheduler.alpha.kubernetes.io/preferAvoidPods": json.dumps({"preferAvoidPods": [{
        "podSignature": {"podController": {"apiVersion": "v1", "kind": kind, "name": "foo", "uid": uid,
                                           "controller": True}},
        "reason": "some reason", "message": "some message"}]})}


@pytest.mark.parametrize("owner,want", [
    ({"kind": "ReplicationController", "name": "foo", "uid": "abcdef123456", "controller": True}, [0, 10, 10]),
    ({"kind": "RandomController", "name": "foo", "uid": "abcdef123456", "controller": True}, [10, 10, 10]),
    ({"kind": "ReplicationController", "name": "foo", "uid": "abcdef123456"}, [10, 10, 10]),
    ({"kind": "ReplicaSet", "name": "foo", "uid": "qwert12345", "controller": True}, [10, 0, 10]),
])
def test_node_prefer_avoid_pods(owner, want):
    cache = SchedulerCache()
    for name, ann in (("machine1", _avoid("ReplicationController", "abcdef123456")),
                      ("machine2", _avoid("ReplicaSet", "qwert12345")), ("machine3", None)):
        n = _node(name, 4000, 10000)
        if ann:
            n["metadata"]["annotations"] = ann
        cache.add_node(n)
    pod = _pod([])
    pod["metadata"]["ownerReferences"] = [dict(owner, apiVersion="v1")]
    gs = GenericScheduler(cache, [], {"NodePreferAvoidPodsPriority": 1}, equivalence_cache=False)
    infos = [cache.nodes[f"machine{i}"] for i in (1, 2, 3)]
    scores = gs.prioritize(pod, PodInfo(pod), infos, CycleContext(cache, pod))
    assert [scores[f"machine{i}"] for i in (1, 2, 3)] == want


# -- resource_limits_test.go ---------------------------------------------------------------------

def _lim(cpu, mem):
    return {"name": "c", "resources": {"limits": {"cpu": cpu, "memory": mem}}}


@pytest.mark.parametrize("ctrs,nodes,want", [
    ([], [(4000, 10000), (4000, 0), (0, 10000), (0, 0)], [0, 0, 0, 0]),
    ([_lim("1000m", "0"), _lim("2000m", "0")], [(3000, 10000), (2000, 10000)], [1, 0]),
    ([_lim("0", "2000"), _lim("0", "3000")], [(4000, 4000), (5000, 10000)], [0, 1]),
    ([_lim("1000m", "2000"), _lim("2000m", "3000")], [(4000, 4000), (5000, 10000)], [1, 1]),
    ([_lim("1000m", "2000"), _lim("2000m", "3000")], [(0, 0)], [0]),
], ids=["no limits", "cpu limits only", "mem limits only", "cpu and mem limits", "zero node"])
def test_resource_limits(ctrs, nodes, want):
    cache = SchedulerCache()
    for i, (cpu, mem) in enumerate(nodes):
        cache.add_node(_node(f"machine{i + 1}", cpu, mem))
    pod = _pod(ctrs)
    gs = GenericScheduler(cache, [], {"ResourceLimitsPriority": 1}, equivalence_cache=False)
    infos = [cache.nodes[f"machine{i + 1}"] for i in range(len(nodes))]
    scores = gs.prioritize(pod, PodInfo(pod), infos, CycleContext(cache, pod))
    assert [scores[f"machine{i + 1}"] for i in range(len(nodes))] == want


# -- interpod_affinity_test.go TestInterPodAffinityPriority / TestHardPodAffinitySymmetricWeight -

S1, S2 = {"security": "S1"}, {"security": "S2"}
RG_CN, RG_IN, AZ1, AZ2 = {"region": "China"}, {"region": "India"}, {"az": "az1"}, {"az": "az2"}
RG_CN_AZ1 = {"region": "China", "az": "az1"}


def _wterm(weight, key, *exprs):
    return {"weight": weight, "podAffinityTerm": {"labelSelector": {"matchExpressions": [
        {"key": k, "operator": op, **({"values": v} if v is not None else {})} for k, op, v in exprs]},
        "topologyKey": key}}


STAY_S1_REGION = {"podAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": [
    _wterm(5, "region", ("security", "In", ["S1"]))]}}
STAY_S2_REGION = {"podAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": [
    _wterm(6, "region", ("security", "In", ["S2"]))]}}
AFFINITY3 = {"podAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": [
    _wterm(8, "region", ("security", "NotIn", ["S1"]), ("security", "In", ["S2"])),
    _wterm(2, "region", ("security", "Exists", None), ("wrongkey", "DoesNotExist", None))]}}
HARD = {"podAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
    _wterm(0, "region", ("security", "In", ["S1", "value2"]))["podAffinityTerm"],
    _wterm(0, "region", ("security", "Exists", None), ("wrongkey", "DoesNotExist", None))["podAffinityTerm"]]}}
AWAY_S1_AZ = {"podAntiAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": [
    _wterm(5, "az", ("security", "In", ["S1"]))]}}
AWAY_S2_AZ = {"podAntiAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": [
    _wterm(5, "az", ("security", "In", ["S2"]))]}}
STAY_S1_AWAY_S2 = {"podAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": [
    _wterm(8, "region", ("security", "In", ["S1"]))]},
    "podAntiAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": [
        _wterm(5, "az", ("security", "In", ["S2"]))]}}


def _ap(labels=None, node=None, affinity=None, i=0):
    spec = {"containers": [{"name": "c"}]}
    if node:
        spec["nodeName"] = node
    if affinity:
        spec["affinity"] = affinity
    return {"metadata": {"name": f"a{i}", "namespace": "default", "uid": f"a{i}", "labels": labels or {}},
            "spec": spec, "status": {"phase": "Running"}}


IPA_CASES = [
    ("affinity is nil", _ap(S1), [], [RG_CN, RG_IN, AZ1], [0, 0, 0]),
    ("matches topology key and pods", _ap(S1, affinity=STAY_S1_REGION),
     [(S1, "machine1", None), (S2, "machine2", None), (S1, "machine3", None)], [RG_CN, RG_IN, AZ1], [10, 0, 0]),
    ("same topology value, same score", _ap(None, affinity=STAY_S1_REGION), [(S1, "machine1", None)],
     [RG_CN, RG_CN_AZ1, RG_IN], [10, 10, 0]),
    ("region with more matches scores higher", _ap(S1, affinity=STAY_S2_REGION),
     [(S2, "machine1", None), (S2, "machine1", None), (S2, "machine2", None), (S2, "machine3", None),
      (S2, "machine4", None), (S2, "machine5", None)], [RG_CN, RG_IN, RG_CN, RG_CN, RG_IN], [10, 5, 10, 10, 5]),
    ("different label operators", _ap(S1, affinity=AFFINITY3),
     [(S1, "machine1", None), (S2, "machine2", None), (S1, "machine3", None)], [RG_CN, RG_IN, AZ1], [2, 10, 0]),
    ("symmetry of preferred affinity", _ap(S2),
     [(S1, "machine1", STAY_S1_REGION), (S2, "machine2", STAY_S2_REGION)], [RG_CN, RG_IN, AZ1], [0, 10, 0]),
    ("symmetry of required affinity", _ap(S1),
     [(S1, "machine1", HARD), (S2, "machine2", HARD)], [RG_CN, RG_IN, AZ1], [10, 10, 0]),
    ("anti affinity: no matching pods scores high", _ap(S1, affinity=AWAY_S1_AZ),
     [(S1, "machine1", None), (S2, "machine2", None)], [AZ1, RG_CN], [0, 10]),
    ("anti affinity: topology key missing scores high", _ap(S1, affinity=AWAY_S1_AZ),
     [(S1, "machine1", None), (S1, "machine2", None)], [AZ1, RG_CN], [0, 10]),
    ("anti affinity: more matches scores low", _ap(S1, affinity=AWAY_S1_AZ),
     [(S1, "machine1", None), (S1, "machine1", None), (S2, "machine2", None)], [AZ1, RG_IN], [0, 10]),
    ("anti affinity symmetry", _ap(S2), [(S1, "machine1", AWAY_S2_AZ), (S2, "machine2", AWAY_S1_AZ)], [AZ1, AZ2],
     [0, 10]),
    ("affinity and anti affinity", _ap(S1, affinity=STAY_S1_AWAY_S2),
     [(S1, "machine1", None), (S1, "machine2", None)], [RG_CN, AZ1], [10, 0]),
    ("affinity and anti affinity, same labels", _ap(S1, affinity=STAY_S1_AWAY_S2),
     [(S1, "machine1", None), (S1, "machine1", None), (S1, "machine2", None), (S1, "machine3", None),
      (S1, "machine3", None), (S1, "machine4", None), (S1, "machine5", None)],
     [RG_CN_AZ1, RG_IN, RG_CN, RG_CN, RG_IN], [10, 4, 10, 10, 4]),
    ("affinity, anti affinity and symmetry", _ap(S1, affinity=STAY_S1_AWAY_S2),
     [(S1, "machine1", None), (S2, "machine2", None), (None, "machine3", STAY_S1_AWAY_S2),
      (None, "machine4", AWAY_S1_AZ)], [RG_CN, AZ1, RG_IN, AZ2], [10, 0, 10, 0]),
]


def _ipa_scores(pod, pods, node_labels, hard_weight=1):
    cache = SchedulerCache()
    cache.hard_pod_affinity_weight = hard_weight
    for i, labels in enumerate(node_labels):
        n = _node(f"machine{i + 1}", 4000, 10000)
        n["metadata"]["labels"] = labels
        cache.add_node(n)
    for i, (labels, node, aff) in enumerate(pods):
        cache.add_pod(_ap(labels, node, aff, i + 1))
    gs = GenericScheduler(cache, [], {"InterPodAffinityPriority": 1}, equivalence_cache=False)
    infos = [cache.nodes[f"machine{i + 1}"] for i in range(len(node_labels))]
    scores = gs.prioritize(pod, PodInfo(pod), infos, CycleContext(cache, pod))
    return [int(scores[f"machine{i + 1}"]) for i in range(len(node_labels))]


@pytest.mark.parametrize("name,pod,pods,node_labels,want", IPA_CASES, ids=[c[0] for c in IPA_CASES])
def test_inter_pod_affinity_priority(name, pod, pods, node_labels, want):
    assert _ipa_scores(pod, pods, node_labels) == want


@pytest.mark.parametrize("weight,want", [(1, [10, 10, 0]), (0, [0, 0, 0])])
def test_hard_pod_affinity_symmetric_weight(weight, want):
    hard = {"podAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
        {"labelSelector": {"matchExpressions": [{"key": "service", "operator": "In", "values": ["S1"]}]},
         "topologyKey": "region"}]}}
    got = _ipa_scores(_ap({"service": "S1"}), [(None, "machine1", hard), (None, "machine2", hard)],
                      [RG_CN, RG_IN, AZ1], hard_weight=weight)
    assert got == want


# -- node_label_test.go TestNewNodeLabelPriority (Policy labelPreference) ------------------------

@pytest.mark.parametrize("label,presence,want", [
    ("baz", True, [0, 0, 0]), ("baz", False, [10, 10, 10]), ("foo", True, [10, 0, 0]), ("foo", False, [0, 10, 10]),
    ("bar", True, [0, 10, 10]), ("bar", False, [10, 0, 0])])
def test_node_label_priority(label, presence, want):
    from kubernetes_amd.scheduler import priorities as PR
    cache = SchedulerCache()
    for i, labels in enumerate(({"foo": "bar"}, {"bar": "foo"}, {"bar": "baz"})):
        n = _node(f"machine{i + 1}", 4000, 10000)
        n["metadata"]["labels"] = labels
        cache.add_node(n)
    pod = _pod([])
    gs = GenericScheduler(cache, [], {"label": (1, PR.make_label_preference(label, presence), False, False)},
                          equivalence_cache=False)
    infos = [cache.nodes[f"machine{i}"] for i in (1, 2, 3)]
    scores = gs.prioritize(pod, PodInfo(pod), infos, CycleContext(cache, pod))
    assert [scores[f"machine{i}"] for i in (1, 2, 3)] == want


# -- taint_toleration_test.go / node_affinity_test.go --------------------------------------------

def _prioritize(prio, pod, nodes):
    cache = SchedulerCache()
    for n in nodes:
        cache.add_node(n)
    gs = GenericScheduler(cache, [], {prio: 1}, equivalence_cache=False)
    infos = [cache.nodes[n["metadata"]["name"]] for n in nodes]
    scores = gs.prioritize(pod, PodInfo(pod), infos, CycleContext(cache, pod))
    return [scores[n["metadata"]["name"]] for n in nodes]


def _tnode(name, taints=(), labels=None):
    n = _node(name, 4000, 10000)
    n["spec"]["taints"] = [{"key": k, "value": v, "effect": e} for k, v, e in taints]
    n["metadata"]["labels"] = dict(labels or {})
    return n


def _tpod(tolerations=(), affinity=None):
    p = _pod([])
    p["spec"]["tolerations"] = [{"key": k, "operator": "Equal", "value": v, "effect": e} for k, v, e in tolerations]
    if affinity:
        p["spec"]["affinity"] = affinity
    return p


PNS, NS = "PreferNoSchedule", "NoSchedule"
CPU, DISK = ("cpu-type", "arm64", PNS), ("disk-type", "ssd", PNS)


@pytest.mark.parametrize("tolerations,nodes,want", [
    # node with taints tolerated by the pod gets a higher score than those with intolerable taints
    ([("foo", "bar", PNS)], [("nodeA", [("foo", "bar", PNS)]), ("nodeB", [("foo", "blah", PNS)])], [10, 0]),
    # the count of tolerated taints does not matter
    ([CPU, DISK], [("nodeA", []), ("nodeB", [CPU]), ("nodeC", [CPU, DISK])], [10, 10, 10]),
    # the more intolerable taints, the lower the score
    ([("foo", "bar", PNS)], [("nodeA", []), ("nodeB", [CPU]), ("nodeC", [CPU, DISK])], [10, 5, 0]),
    # only PreferNoSchedule taints and tolerations count
    ([("cpu-type", "arm64", NS), ("disk-type", "ssd", NS)],
     [("nodeA", []), ("nodeB", [("cpu-type", "arm64", NS)]), ("nodeC", [CPU, DISK])], [10, 10, 0]),
    # default: no taints and tolerations, lands on the node without taints
    ([], [("nodeA", []), ("nodeB", [CPU])], [10, 0]),
])
def test_taint_and_toleration(tolerations, nodes, want):
    assert _prioritize("TaintTolerationPriority", _tpod(tolerations), [_tnode(n, t) for n, t in nodes]) == want


def _pref(weight, *exprs):
    return {"weight": weight, "preference": {"matchExpressions": [
        {"key": k, "operator": "In", "values": [v]} for k, v in exprs]}}


AFF1 = {"nodeAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": [_pref(2, ("foo", "bar"))]}}
AFF2 = {"nodeAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": [
    _pref(2, ("foo", "bar")), _pref(4, ("key", "value")), _pref(5, ("foo", "bar"), ("key", "value"), ("az", "az1"))]}}
L1, L2, L3 = {"foo": "bar"}, {"key": "value"}, {"az": "az1"}
L4, L5 = {"abc": "az11", "def": "az22"}, {"foo": "bar", "key": "value", "az": "az1"}


@pytest.mark.parametrize("affinity,nodes,want", [
    (None, [("machine1", L1), ("machine2", L2), ("machine3", L3)], [0, 0, 0]),
    (AFF1, [("machine1", L4), ("machine2", L2), ("machine3", L3)], [0, 0, 0]),
    (AFF1, [("machine1", L1), ("machine2", L2), ("machine3", L3)], [10, 0, 0]),
    (AFF2, [("machine1", L1), ("machine5", L5), ("machine2", L2)], [1, 10, 3]),
])
def test_node_affinity_priority(affinity, nodes, want):
    assert _prioritize("NodeAffinityPriority", _tpod(affinity=affinity), [_tnode(n, labels=lb) for n, lb in nodes]) == want
