"""Ported generic-scheduler tables.

Reference: `plugin/pkg/scheduler/core/generic_scheduler_test.go` — TestSelectHost (:117),
TestGenericScheduler (:183, tests 1-8), TestFindFitAllError / TestFindFitSomeError (:326-408),
TestHumanReadableFitError (:410), TestZeroRequest (:433). Function-style priorities that see the
whole node list (`reverseNumericPriority`) use a callable reduce step. SelectorSpreadPriority is
skipped for a pod with no owner and no service (every node would score 10): TestZeroRequest's
expected 25 is therefore 15 here — the same ranking, shifted by a constant.
"""
import pytest

from kubernetes_amd.scheduler.cache import PodInfo, SchedulerCache
from kubernetes_amd.scheduler.generic import CycleContext, FitError, GenericScheduler

FAKE = "FakePredicateError"


def false_pred(pod, pi, ni, ctx):
    return FAKE


def true_pred(pod, pi, ni, ctx):
    return None


def matches_pred(pod, pi, ni, ctx):
    return None if pod["metadata"]["name"] == ni.name else FAKE


def has_no_pods_pred(pod, pi, ni, ctx):
    return None if not ni.pods else FAKE


def numeric(pod, pi, ni, ctx):
    return int(ni.name)


def reverse_reduce(col, nodes):
    """reverseNumericPriority: max + min - score over the feasible nodes."""
    return [max(col) + min(col) - s for s in col]


NUMERIC = ("numeric", (1, numeric, False, None))
REVERSE2 = ("reverse", (2, numeric, False, reverse_reduce))
EQUAL = ("EqualPriority", 1)


def _node(name, cpu_m=None, mem=None):
    alloc = {"pods": "100"}
    if cpu_m is not None:
        alloc.update(cpu=f"{cpu_m}m", memory=str(mem))
    else:
        alloc.update(cpu="4", memory="8Gi")
    return {"metadata": {"name": name}, "spec": {},
            "status": {"allocatable": alloc, "capacity": dict(alloc), "conditions": [{"type": "Ready", "status": "True"}]}}


def _pod(name, node=None, requests=None):
    c = {"name": "c", "image": "x"}
    if requests:
        c["resources"] = {"requests": requests}
    spec = {"containers": [c]}
    if node:
        spec["nodeName"] = node
    return {"metadata": {"name": name, "namespace": "default", "uid": f"u-{name}-{node}"}, "spec": spec,
            "status": {"phase": "Running"}}


CASES = [
    ("test 1", [("false", false_pred)], [EQUAL], ["machine1", "machine2"], "2", [], None,
     {"machine1": FAKE, "machine2": FAKE}),
    ("test 2", [("true", true_pred)], [EQUAL], ["machine1", "machine2"], "ignore", [], {"machine1", "machine2"}, None),
    ("test 3", [("matches", matches_pred)], [EQUAL], ["machine1", "machine2"], "machine2", [], {"machine2"}, None),
    ("test 4", [("true", true_pred)], [NUMERIC], ["3", "2", "1"], "ignore", [], {"3"}, None),
    ("test 5", [("matches", matches_pred)], [NUMERIC], ["3", "2", "1"], "2", [], {"2"}, None),
    ("test 6", [("true", true_pred)], [NUMERIC, REVERSE2], ["3", "2", "1"], "2", [], {"1"}, None),
    ("test 7", [("true", true_pred), ("false", false_pred)], [NUMERIC], ["3", "2", "1"], "2", [], None,
     {"3": FAKE, "2": FAKE, "1": FAKE}),
    ("test 8", [("nopods", has_no_pods_pred), ("matches", matches_pred)], [NUMERIC], ["1", "2"], "2",
     [_pod("2", node="2")], None, {"1": FAKE, "2": FAKE}),
]


@pytest.mark.parametrize("name,preds,prios,nodes,pod_name,pods,expected,want_failed", CASES, ids=[c[0] for c in CASES])
def test_generic_scheduler(name, preds, prios, nodes, pod_name, pods, expected, want_failed):
    cache = SchedulerCache()
    for n in nodes:
        cache.add_node(_node(n))
    for p in pods:
        cache.add_pod(p)
    gs = GenericScheduler(cache, preds, dict(prios), equivalence_cache=False)
    pod = _pod(pod_name)
    if want_failed is not None:
        with pytest.raises(FitError) as e:
            gs.schedule(pod)
        assert e.value.num_nodes == len(nodes)
        assert e.value.failed == want_failed
    else:
        for _ in range(4):       # ties rotate; every answer must be an expected host
            host, _ = gs.schedule(pod)
            assert host in expected, name


@pytest.mark.parametrize("scores,possible", [
    ({"machine1.1": 1, "machine2.1": 2}, {"machine2.1"}),
    ({"machine1.1": 1, "machine1.2": 2, "machine1.3": 2, "machine2.1": 2}, {"machine1.2", "machine1.3", "machine2.1"}),
    ({"machine1.1": 3, "machine1.2": 3, "machine2.1": 2, "machine3.1": 1, "machine1.3": 3},
     {"machine1.1", "machine1.2", "machine1.3"}),
])
def test_select_host(scores, possible):
    gs = GenericScheduler(SchedulerCache(), [], {})

    class N:
        def __init__(self, name):
            self.name = name
    nodes = [N(n) for n in scores]
    seen = {gs.select_host(scores, nodes) for _ in range(10)}
    assert seen <= possible
    if len(possible) > 1:
        assert len(seen) > 1            # equal scores are spread round-robin


def test_select_host_empty_list_is_an_error():
    with pytest.raises(ValueError):
        GenericScheduler(SchedulerCache(), [], {}).select_host({}, [])


def test_find_fit_all_error_and_some_error():
    cache = SchedulerCache()
    for n in ("3", "2", "1"):
        cache.add_node(_node(n))
    gs = GenericScheduler(cache, [("true", true_pred), ("false", false_pred)], {}, equivalence_cache=False)
    with pytest.raises(FitError) as e:
        gs.schedule(_pod("x"))
    assert e.value.failed == {"3": FAKE, "2": FAKE, "1": FAKE}
    # TestFindFitSomeError: only node "1" matches; the other two report the fake predicate
    gs = GenericScheduler(cache, [("true", true_pred), ("match", matches_pred)], {}, equivalence_cache=False)
    host, _ = gs.schedule(_pod("1"))
    assert host == "1"
    gs2 = GenericScheduler(cache, [("match", matches_pred), ("false", false_pred)], {}, equivalence_cache=False)
    with pytest.raises(FitError) as e:
        gs2.schedule(_pod("1"))
    assert set(e.value.failed) == {"1", "2", "3"} and e.value.failed["2"] == FAKE


def test_human_readable_fit_error():
    err = FitError(_pod("2"), 3, {"1": "NodeUnderMemoryPressure", "2": "NodeUnderDiskPressure",
                                  "3": "NodeUnderDiskPressure"})
    s = str(err)
    assert "0/3 nodes are available" in s and "2 NodeUnderDiskPressure" in s and "1 NodeUnderMemoryPressure" in s


DEFAULT_CPU_M, DEFAULT_MEM = 100, 200 * 1024 * 1024


@pytest.mark.parametrize("case", ["zero-request pod", "nonzero-request pod", "larger pod"])
def test_zero_request(case):
    """A zero-request pod counts as the default request (100m, 200Mi) in LeastRequested and
    BalancedResourceAllocation, whether it is being scheduled or already on the node."""
    small = {"cpu": f"{DEFAULT_CPU_M}m", "memory": str(DEFAULT_MEM)}
    large = {"cpu": f"{DEFAULT_CPU_M * 3}m", "memory": str(DEFAULT_MEM * 3)}
    cache = SchedulerCache()
    for n in ("machine1", "machine2"):
        cache.add_node(_node(n, 1000, DEFAULT_MEM * 10))
    for p in (_pod("large1", "machine1", large), _pod("zero1", "machine1"), _pod("large2", "machine2", large),
              _pod("small2", "machine2", small)):
        cache.add_pod(p)
    pod = {"zero-request pod": _pod("new"), "nonzero-request pod": _pod("new", requests=small),
           "larger pod": _pod("new", requests=large)}[case]
    gs = GenericScheduler(cache, [], {"LeastRequestedPriority": 1, "BalancedResourceAllocation": 1,
                                      "SelectorSpreadPriority": 1}, equivalence_cache=False)
    nodes = [cache.nodes["machine1"], cache.nodes["machine2"]]
    scores = gs.prioritize(pod, PodInfo(pod), nodes, CycleContext(cache, pod))
    if case == "larger pod":
        assert all(s != 15 for s in scores.values()), scores
    else:
        assert all(s == 15 for s in scores.values()), scores


# -- predicates_test.go TestPodFitsSelector ------------------------------------------------------

def _req(*terms):
    return {"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {"nodeSelectorTerms": list(terms)}}}


def _term(*exprs):
    return {"matchExpressions": [dict(zip(("key", "operator", "values"), e)) if len(e) == 3 else
                                 {"key": e[0], "operator": e[1]} for e in exprs]}


SELECTOR_CASES = [
    ("no selector", {}, {}, True),
    ("missing labels", {"nodeSelector": {"foo": "bar"}}, {}, False),
    ("same labels", {"nodeSelector": {"foo": "bar"}}, {"foo": "bar"}, True),
    ("node labels are superset", {"nodeSelector": {"foo": "bar"}}, {"foo": "bar", "baz": "blah"}, True),
    ("node labels are subset", {"nodeSelector": {"foo": "bar", "baz": "blah"}}, {"foo": "bar"}, False),
    ("In matches", {"affinity": _req(_term(("foo", "In", ["bar", "value2"])))}, {"foo": "bar"}, True),
    ("Gt matches", {"affinity": _req(_term(("kernel-version", "Gt", ["0204"])))}, {"kernel-version": "0206"}, True),
    ("NotIn matches", {"affinity": _req(_term(("mem-type", "NotIn", ["DDR", "DDR2"])))}, {"mem-type": "DDR3"}, True),
    ("Exists matches", {"affinity": _req(_term(("GPU", "Exists")))}, {"GPU": "NVIDIA-GRID-K1"}, True),
    ("affinity does not match", {"affinity": _req(_term(("foo", "In", ["value1", "value2"])))}, {"foo": "bar"}, False),
    ("nil NodeSelectorTerms", {"affinity": {"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {}}}},
     {"foo": "bar"}, False),
    ("empty NodeSelectorTerms", {"affinity": _req()}, {"foo": "bar"}, False),
    ("empty MatchExpressions", {"affinity": _req({"matchExpressions": []})}, {"foo": "bar"}, False),
    ("no Affinity", {}, {"foo": "bar"}, True),
    ("Affinity but nil NodeSelector", {"affinity": {"nodeAffinity": {}}}, {"foo": "bar"}, True),
    ("multiple matchExpressions ANDed, match",
     {"affinity": _req(_term(("GPU", "Exists"), ("GPU", "NotIn", ["AMD", "INTER"])))}, {"GPU": "NVIDIA-GRID-K1"}, True),
    ("multiple matchExpressions ANDed, no match",
     {"affinity": _req(_term(("GPU", "Exists"), ("GPU", "In", ["AMD", "INTER"])))}, {"GPU": "NVIDIA-GRID-K1"}, False),
    ("multiple NodeSelectorTerms ORed",
     {"affinity": _req(_term(("foo", "In", ["bar", "value2"])), _term(("diffkey", "In", ["wrong", "value2"])))},
     {"foo": "bar"}, True),
    ("Affinity and NodeSelector both satisfied",
     {"nodeSelector": {"foo": "bar"}, "affinity": _req(_term(("foo", "Exists")))}, {"foo": "bar"}, True),
    ("Affinity matches but NodeSelector does not",
     {"nodeSelector": {"foo": "bar"}, "affinity": _req(_term(("foo", "Exists")))}, {"foo": "barrrrrr"}, False),
]


@pytest.mark.parametrize("name,spec,labels,fits", SELECTOR_CASES, ids=[c[0] for c in SELECTOR_CASES])
def test_pod_fits_selector(name, spec, labels, fits):
    from kubernetes_amd.scheduler.predicates import match_node_selector
    cache = SchedulerCache()
    node = _node("machine1")
    node["metadata"]["labels"] = labels
    cache.add_node(node)
    pod = {"metadata": {"name": "p", "namespace": "default"}, "spec": dict(spec, containers=[{"name": "c"}])}
    got = match_node_selector(pod, PodInfo(pod), cache.nodes["machine1"], None)
    assert (got is None) == fits, (name, got)


# -- predicates_test.go TestInterPodAffinity -----------------------------------------------------

SEC = {"service": "securityscan"}
SEC2 = {"security": "S1"}


def _sel(*exprs):
    return {"matchExpressions": [{"key": k, "operator": op, **({"values": v} if v is not None else {})}
                                 for k, op, v in exprs]}


def _aff_term(*exprs, key="region", namespaces=None):
    t = {"labelSelector": _sel(*exprs)}
    if key:
        t["topologyKey"] = key
    if namespaces:
        t["namespaces"] = namespaces
    return t


def _affinity(aff=(), anti=()):
    out = {}
    if aff:
        out["podAffinity"] = {"requiredDuringSchedulingIgnoredDuringExecution": list(aff)}
    if anti:
        out["podAntiAffinity"] = {"requiredDuringSchedulingIgnoredDuringExecution": list(anti)}
    return out


def _apod(name, labels, node=None, affinity=None, ns="default"):
    spec = {"containers": [{"name": "c"}]}
    if node:
        spec["nodeName"] = node
    if affinity:
        spec["affinity"] = affinity
    return {"metadata": {"name": name, "namespace": ns, "uid": f"u-{name}", "labels": labels}, "spec": spec,
            "status": {"phase": "Running"}}


IN_SEC = ("service", "In", ["securityscan", "value2"])
IN_AV = ("service", "In", ["antivirusscan", "value2"])
AFFINITY_CASES = [
    ("no required pod affinity, empty node", _apod("p", {}), [], True),
    ("PodAffinity In matches the existing pod",
     _apod("p", SEC2, affinity=_affinity([_aff_term(IN_SEC)])), [_apod("e", SEC, "machine1")], True),
    ("PodAffinity NotIn matches the existing pod",
     _apod("p", SEC2, affinity=_affinity([_aff_term(("service", "NotIn", ["securityscan3", "value3"]))])),
     [_apod("e", SEC, "machine1")], True),
    ("diff Namespace",
     _apod("p", SEC2, affinity=_affinity([_aff_term(IN_SEC, key="", namespaces=["DiffNameSpace"])])),
     [_apod("e", SEC, "machine1", ns="ns")], False),
    ("unmatching labelSelector", _apod("p", SEC, affinity=_affinity([_aff_term(IN_AV, key="")])),
     [_apod("e", SEC, "machine1")], False),
    ("different label operators in multiple terms",
     _apod("p", SEC2, affinity=_affinity([_aff_term(("service", "Exists", None), ("wrongkey", "DoesNotExist", None)),
                                          _aff_term(("service", "In", ["securityscan"]),
                                                    ("service", "NotIn", ["WrongValue"]))])),
     [_apod("e", SEC, "machine1")], True),
    ("matchExpressions are ANDed",
     _apod("p", SEC2, affinity=_affinity([_aff_term(("service", "Exists", None), ("wrongkey", "DoesNotExist", None)),
                                          _aff_term(("service", "In", ["securityscan2"]),
                                                    ("service", "NotIn", ["WrongValue"]))])),
     [_apod("e", SEC, "machine1")], False),
    ("PodAffinity and PodAntiAffinity",
     _apod("p", SEC2, affinity=_affinity([_aff_term(IN_SEC)], [_aff_term(IN_AV, key="node")])),
     [_apod("e", SEC, "machine1")], True),
    ("PodAffinity, PodAntiAffinity and symmetry",
     _apod("p", SEC2, affinity=_affinity([_aff_term(IN_SEC)], [_aff_term(IN_AV, key="node")])),
     [_apod("e", SEC, "machine1", affinity=_affinity(anti=[_aff_term(IN_AV, key="node")]))], True),
    ("PodAffinity but not PodAntiAffinity",
     _apod("p", SEC2, affinity=_affinity([_aff_term(IN_SEC)], [_aff_term(IN_SEC, key="zone")])),
     [_apod("e", SEC, "machine1")], False),
    ("existing pod's anti-affinity symmetry violated",
     _apod("p", SEC, affinity=_affinity([_aff_term(IN_SEC)], [_aff_term(IN_AV, key="node")])),
     [_apod("e", SEC, "machine1", affinity=_affinity(anti=[_aff_term(IN_SEC, key="zone")]))], False),
    ("pod matches its own label NotIn",
     _apod("p", SEC, affinity=_affinity([_aff_term(("service", "NotIn", ["securityscan", "value2"]))])),
     [_apod("e", SEC, "machine2")], False),
    ("existing pod anti-affinity respected without own constraints",
     _apod("p", SEC), [_apod("e", SEC, "machine1", affinity=_affinity(anti=[_aff_term(IN_SEC, key="zone")]))], False),
    ("existing pod anti-affinity satisfied without own constraints",
     _apod("p", SEC), [_apod("e", SEC, "machine1", affinity=_affinity(
         anti=[_aff_term(("service", "NotIn", ["securityscan", "value2"]), key="zone")]))], True),
]


@pytest.mark.parametrize("name,pod,pods,fits", AFFINITY_CASES, ids=[c[0] for c in AFFINITY_CASES])
def test_inter_pod_affinity(name, pod, pods, fits):
    from kubernetes_amd.scheduler.predicates import match_inter_pod_affinity
    cache = SchedulerCache()
    node = _node("machine1")
    node["metadata"]["labels"] = {"region": "r1", "zone": "z11"}
    cache.add_node(node)
    for p in pods:
        cache.add_pod(p)
    got = match_inter_pod_affinity(pod, PodInfo(pod), cache.nodes["machine1"], CycleContext(cache, pod))
    assert (got is None) == fits, (name, got)


# -- predicates_test.go TestInterPodAffinityWithMultipleNodes ------------------------------------

CN, CN_AZ, IN_, US = {"region": "China"}, {"region": "China", "az": "az1"}, {"region": "India"}, {"region": "US"}
MULTI_CASES = [
    ("same topology value as a node with a matching pod",
     _apod("p", {}, affinity=_affinity([_aff_term(("foo", "In", ["bar"]))])),
     [_apod("e", {"foo": "bar"}, "machine1")], [("machine1", CN), ("machine2", CN_AZ), ("machine3", IN_)],
     {"machine1": True, "machine2": True, "machine3": False}),
    ("node affinity excludes nodeA, pod affinity satisfied through nodeB's region",
     dict(_apod("p", {}, affinity=dict(_affinity([_aff_term(("foo", "In", ["abc"]))]),
                                        **_req(_term(("hostname", "NotIn", ["h1"])))))),
     [_apod("a", {"foo": "abc"}, "nodeA"), _apod("b", {"foo": "def"}, "nodeB")],
     [("nodeA", {"region": "r1", "hostname": "h1"}), ("nodeB", {"region": "r1", "hostname": "h2"})],
     {"nodeA": False, "nodeB": True}),
    ("first pod of a collection may go anywhere",
     _apod("p", {"foo": "bar"}, affinity=_affinity([_aff_term(("foo", "In", ["bar"]), key="zone")])), [],
     [("nodeA", {"zone": "az1", "hostname": "h1"}), ("nodeB", {"zone": "az2", "hostname": "h2"})],
     {"nodeA": True, "nodeB": True}),
    ("anti-affinity blocks the whole region",
     _apod("p", {}, affinity=_affinity(anti=[_aff_term(("foo", "In", ["abc"]))])), [_apod("a", {"foo": "abc"}, "nodeA")],
     [("nodeA", {"region": "r1", "hostname": "nodeA"}), ("nodeB", {"region": "r1", "hostname": "nodeB"})],
     {"nodeA": False, "nodeB": False}),
    ("anti-affinity blocks China, India is free",
     _apod("p", {}, affinity=_affinity(anti=[_aff_term(("foo", "In", ["abc"]))])), [_apod("a", {"foo": "abc"}, "nodeA")],
     [("nodeA", CN), ("nodeB", CN_AZ), ("nodeC", IN_)], {"nodeA": False, "nodeB": False, "nodeC": True}),
    ("own anti-affinity plus an existing pod's anti-affinity",
     _apod("p", {"foo": "123"}, affinity=_affinity(anti=[_aff_term(("foo", "In", ["bar"]))])),
     [_apod("a", {"foo": "bar"}, "nodeA"),
      _apod("c", {}, "nodeC", affinity=_affinity(anti=[_aff_term(("foo", "In", ["123"]))]))],
     [("nodeA", CN), ("nodeB", CN_AZ), ("nodeC", IN_), ("nodeD", US)],
     {"nodeA": False, "nodeB": False, "nodeC": False, "nodeD": True}),
    ("an existing pod's anti-affinity in another namespace does not apply",
     _apod("p", {"foo": "123"}, ns="NS1", affinity=_affinity(anti=[_aff_term(("foo", "In", ["bar"]))])),
     [_apod("a", {"foo": "bar"}, "nodeA", ns="NS1"),
      _apod("c", {}, "nodeC", ns="NS2", affinity=_affinity(anti=[_aff_term(("foo", "In", ["123"]))]))],
     [("nodeA", CN), ("nodeB", CN_AZ), ("nodeC", IN_)], {"nodeA": False, "nodeB": False, "nodeC": True}),
]


@pytest.mark.parametrize("name,pod,pods,nodes,fits", MULTI_CASES, ids=[c[0] for c in MULTI_CASES])
def test_inter_pod_affinity_with_multiple_nodes(name, pod, pods, nodes, fits):
    from kubernetes_amd.scheduler.predicates import match_inter_pod_affinity, match_node_selector
    cache = SchedulerCache()
    for n, labels in nodes:
        node = _node(n)
        node["metadata"]["labels"] = labels
        cache.add_node(node)
    for p in pods:
        cache.add_pod(p)
    ctx = CycleContext(cache, pod)
    for n, _ in nodes:
        ni = cache.nodes[n]
        ok = match_inter_pod_affinity(pod, PodInfo(pod), ni, ctx) is None and \
            match_node_selector(pod, PodInfo(pod), ni, ctx) is None
        assert ok == fits[n], (name, n)


# -- predicates_test.go TestPodToleratesTaints / pressure conditions / TestNodeConditionPredicate -

def _tol(key, value=None, effect=None, op=None):
    t = {"key": key}
    for k, v in (("value", value), ("effect", effect), ("operator", op)):
        if v is not None:
            t[k] = v
    return t


TAINT_CASES = [
    ("no tolerations vs taint", [], [{"key": "dedicated", "value": "user1", "effect": "NoSchedule"}], False),
    ("dedicated to user1", [_tol("dedicated", "user1", "NoSchedule")],
     [{"key": "dedicated", "value": "user1", "effect": "NoSchedule"}], True),
    ("dedicated to user2", [_tol("dedicated", "user2", "NoSchedule", "Equal")],
     [{"key": "dedicated", "value": "user1", "effect": "NoSchedule"}], False),
    ("Exists tolerates", [_tol("foo", None, "NoSchedule", "Exists")],
     [{"key": "foo", "value": "bar", "effect": "NoSchedule"}], True),
    ("all taints tolerated", [_tol("dedicated", "user2", "NoSchedule", "Equal"), _tol("foo", None, "NoSchedule", "Exists")],
     [{"key": "dedicated", "value": "user2", "effect": "NoSchedule"}, {"key": "foo", "value": "bar", "effect": "NoSchedule"}],
     True),
    ("non-empty effect mismatch", [_tol("foo", "bar", "PreferNoSchedule", "Equal")],
     [{"key": "foo", "value": "bar", "effect": "NoSchedule"}], False),
    ("empty effect tolerates all effects", [_tol("foo", "bar", None, "Equal")],
     [{"key": "foo", "value": "bar", "effect": "NoSchedule"}], True),
    ("PreferNoSchedule is not enforced", [_tol("dedicated", "user2", "NoSchedule", "Equal")],
     [{"key": "dedicated", "value": "user1", "effect": "PreferNoSchedule"}], True),
    ("no toleration, only PreferNoSchedule", [], [{"key": "dedicated", "value": "user1", "effect": "PreferNoSchedule"}],
     True),
]


@pytest.mark.parametrize("name,tols,taints,fits", TAINT_CASES, ids=[c[0] for c in TAINT_CASES])
def test_pod_tolerates_taints(name, tols, taints, fits):
    from kubernetes_amd.scheduler.predicates import pod_tolerates_node_taints
    cache = SchedulerCache()
    node = _node("n")
    node["spec"]["taints"] = taints
    cache.add_node(node)
    pod = {"metadata": {"name": "p", "namespace": "default"}, "spec": {"containers": [{"name": "c"}],
                                                                       "tolerations": tols}}
    assert (pod_tolerates_node_taints(pod, PodInfo(pod), cache.nodes["n"], None) is None) == fits


@pytest.mark.parametrize("best_effort,pressure,fits", [(True, False, True), (True, True, False), (False, True, True),
                                                       (False, False, True)])
def test_memory_pressure(best_effort, pressure, fits):
    from kubernetes_amd.scheduler.predicates import check_node_memory_pressure
    cache = SchedulerCache()
    node = _node("n")
    node["status"]["conditions"].append({"type": "MemoryPressure", "status": "True" if pressure else "False"})
    cache.add_node(node)
    pod = _pod("p", requests=None if best_effort else {"cpu": "100m", "memory": "100"})
    assert (check_node_memory_pressure(pod, PodInfo(pod), cache.nodes["n"], None) is None) == fits


@pytest.mark.parametrize("pressure,fits", [(False, True), (True, False)])
def test_disk_pressure(pressure, fits):
    from kubernetes_amd.scheduler.predicates import check_node_disk_pressure
    cache = SchedulerCache()
    node = _node("n")
    node["status"]["conditions"].append({"type": "DiskPressure", "status": "True" if pressure else "False"})
    cache.add_node(node)
    pod = _pod("p")
    assert (check_node_disk_pressure(pod, PodInfo(pod), cache.nodes["n"], None) is None) == fits


@pytest.mark.parametrize("conditions,unschedulable,fits", [
    ([("Ready", "True")], False, True), ([("Ready", "False")], False, False), ([("OutOfDisk", "True")], False, False),
    ([("OutOfDisk", "False")], False, True), ([("Ready", "True"), ("OutOfDisk", "True")], False, False),
    ([("Ready", "True"), ("OutOfDisk", "False")], False, True), ([("Ready", "False"), ("OutOfDisk", "True")], False, False),
    ([("Ready", "False"), ("OutOfDisk", "False")], False, False), ([], True, False), ([], False, True),
    ([("Ready", "True"), ("NetworkUnavailable", "True")], False, False),
])
def test_node_condition_predicate(conditions, unschedulable, fits):
    from kubernetes_amd.scheduler.predicates import check_node_condition
    cache = SchedulerCache()
    node = {"metadata": {"name": "n"}, "spec": {"unschedulable": unschedulable},
            "status": {"allocatable": {"cpu": "1", "memory": "1Gi", "pods": "10"},
                       "conditions": [{"type": t, "status": s} for t, s in conditions]}}
    cache.add_node(node)
    pod = _pod("p")
    assert (check_node_condition(pod, PodInfo(pod), cache.nodes["n"], CycleContext(cache, pod)) is None) == fits


def test_pod_backoff():
    """`plugin/pkg/scheduler/util/backoff_utils_test.go` TestBackoff."""
    from kubernetes_amd.scheduler.queue import PodBackoff
    now = [0.0]
    b = PodBackoff(1.0, 60.0, clock=lambda: now[0])
    for key, want, advance in (("default/foo", 1, 0), ("default/foo", 2, 0), ("default/foo", 4, 0),
                               ("default/bar", 1, 120), ("default/foo", 1, 0)):      # foo gc'd after 120 s
        assert b.next(key) == want, key
        now[0] += advance
        b.gc()
    b.entries["default/foo"] = 60.0
    assert b.next("default/foo") == 60.0                                            # capped
