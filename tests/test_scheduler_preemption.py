"""Ported preemption and nominated-pod tables.

Reference: `plugin/pkg/scheduler/core/generic_scheduler_test.go` TestSelectNodesForPreemption
(:666-801), TestPickOneNodeForPreemption (:804-963), TestNodesWherePreemptionMightHelp
(:965-1081), TestPreempt (:1083-1215); `plugin/pkg/scheduler/core/scheduling_queue_test.go`
(:89-321). Node capacity is 5 × (100m, 200Mi) as in the reference's `makeNode`. The GPU cases at
the end are MI355X additions: nominees hold device IDs, PDB-aware victims, eligibility.
"""
from kubernetes_amd.api import core
from kubernetes_amd.scheduler import predicates as P
from kubernetes_amd.scheduler.cache import PodInfo, SchedulerCache
from kubernetes_amd.scheduler.generic import FitError, GenericScheduler
from kubernetes_amd.scheduler.preemption import (NOMINATED_ANNOTATION, Victims, nodes_where_preemption_might_help,
                                                 pick_one_node_for_preemption, pod_eligible_to_preempt_others,
                                                 preempt, select_nodes_for_preemption, select_victims_on_node)
from kubernetes_amd.scheduler.queue import SchedulingQueue

from test_scheduler import gpu_dev, gpu_pod, node as gpu_node

NEG, LOW, MID, HIGH, VHIGH = -100, 0, 100, 1000, 10000
CPU, MEM = 100, 200 * 1024 * 1024


def ctrs(mult):
    return [{"name": "c", "image": "x", "resources": {"requests": {"cpu": f"{CPU * mult}m", "memory": str(MEM * mult)}}}]


SMALL, MEDIUM, LARGE, VLARGE = ctrs(1), ctrs(2), ctrs(3), ctrs(5)


def pod(name, prio, node=None, containers=None, labels=None, affinity=None, ns="default", annotations=None):
    spec = {"priority": prio, "containers": containers or [{"name": "c", "image": "x"}]}
    if node:
        spec["nodeName"] = node
    if affinity:
        spec["affinity"] = affinity
    md = {"name": name, "namespace": ns, "uid": f"uid-{ns}-{name}"}
    if labels:
        md["labels"] = labels
    if annotations:
        md["annotations"] = annotations
    return {"metadata": md, "spec": spec, "status": {"phase": "Running"}}


def make_node(name):
    return {"metadata": {"name": name, "labels": {"hostname": name}},
            "spec": {}, "status": {"allocatable": {"cpu": f"{CPU * 5}m", "memory": str(MEM * 5), "pods": "100"},
                                   "conditions": [{"type": "Ready", "status": "True"}]}}


def false_pred(pod, pi, ni, ctx):
    return "false"


def true_pred(pod, pi, ni, ctx):
    return None


def matches_pred(pod, pi, ni, ctx):
    return None if pod["metadata"]["name"] == ni.name else "not machine"


def setup(node_names, pods, predicates, extenders=None):
    cache = SchedulerCache()
    for n in node_names:
        cache.add_node(make_node(n))
    for p in pods:
        cache.add_pod(p)
    gs = GenericScheduler(cache, predicates, priorities={}, extenders=extenders, equivalence_cache=False)
    return cache, gs


def names(victims):
    return {p["metadata"]["name"] for p in victims}


ANTI = {"podAntiAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [{
    "labelSelector": {"matchExpressions": [{"key": "pod", "operator": "In", "values": ["preemptor", "value2"]}]},
    "topologyKey": "hostname"}]}}

FITS = ("matches", P.pod_fits_resources)

SELECT_CASES = [
    ("a pod that does not fit on any machine", [("matches", false_pred)], pod("new", HIGH),
     [pod("a", MID, "machine1"), pod("b", MID, "machine2")], {}),
    ("a pod that fits with no preemption", [("matches", true_pred)], pod("new", HIGH),
     [pod("a", MID, "machine1"), pod("b", MID, "machine2")], {"machine1": set(), "machine2": set()}),
    ("a pod that fits on one machine with no preemption", [("matches", matches_pred)], pod("machine1", HIGH),
     [pod("a", MID, "machine1"), pod("b", MID, "machine2")], {"machine1": set()}),
    ("a pod that fits on both machines when lower priority pods are preempted", [FITS],
     pod("machine1", HIGH, containers=LARGE),
     [pod("a", MID, "machine1", LARGE), pod("b", MID, "machine2", LARGE)], {"machine1": {"a"}, "machine2": {"b"}}),
    ("a pod that would fit on the machines, but other pods running are higher priority", [FITS],
     pod("machine1", LOW, containers=LARGE),
     [pod("a", MID, "machine1", LARGE), pod("b", MID, "machine2", LARGE)], {}),
    ("medium priority pod is preempted, but lower priority one stays as it is small", [FITS],
     pod("machine1", HIGH, containers=LARGE),
     [pod("a", LOW, "machine1", SMALL), pod("b", MID, "machine1", LARGE), pod("c", MID, "machine2", LARGE)],
     {"machine1": {"b"}, "machine2": {"c"}}),
    ("mixed priority pods are preempted", [FITS], pod("machine1", HIGH, containers=LARGE),
     [pod("a", MID, "machine1", SMALL), pod("b", LOW, "machine1", SMALL), pod("c", MID, "machine1", MEDIUM),
      pod("d", HIGH, "machine1", SMALL), pod("e", HIGH, "machine2", LARGE)], {"machine1": {"b", "c"}}),
    ("pod with anti-affinity is preempted", [FITS, ("MatchInterPodAffinity", P.match_inter_pod_affinity)],
     pod("machine1", HIGH, containers=SMALL, labels={"pod": "preemptor"}),
     [pod("a", LOW, "machine1", SMALL, labels={"service": "securityscan"}, affinity=ANTI),
      pod("b", MID, "machine1", SMALL), pod("d", HIGH, "machine1", SMALL), pod("e", HIGH, "machine2", LARGE)],
     {"machine1": {"a"}, "machine2": set()}),
]


def test_select_nodes_for_preemption_table():
    for name, preds, p, pods, expected in SELECT_CASES:
        cache, gs = setup(["machine1", "machine2"], pods, preds)
        got = select_nodes_for_preemption(gs, p, PodInfo(p), cache.node_list())
        assert {n: names(v.pods) for n, v in got.items()} == expected, name
        for v in got.values():     # victims are sorted by decreasing priority
            prios = [x["spec"]["priority"] for x in v.pods]
            assert prios == sorted(prios, reverse=True), name


PICK_CASES = [
    ("No node needs preemption", ["machine1"], pod("machine1", HIGH, containers=LARGE),
     [pod("m1.1", MID, "machine1", SMALL)], {"machine1"}),
    ("a pod that fits on both machines when lower priority pods are preempted", ["machine1", "machine2"],
     pod("machine1", HIGH, containers=LARGE),
     [pod("m1.1", MID, "machine1", LARGE), pod("m2.1", MID, "machine2", LARGE)], {"machine1", "machine2"}),
    ("a pod that fits on a machine with no preemption", ["machine1", "machine2", "machine3"],
     pod("machine1", HIGH, containers=LARGE),
     [pod("m1.1", MID, "machine1", LARGE), pod("m2.1", MID, "machine2", LARGE)], {"machine3"}),
    ("machine with min highest priority pod is picked", ["machine1", "machine2", "machine3"],
     pod("machine1", HIGH, containers=VLARGE),
     [pod("m1.1", MID, "machine1", MEDIUM), pod("m1.2", MID, "machine1", LARGE),
      pod("m2.1", MID, "machine2", MEDIUM), pod("m2.2", LOW, "machine2", MEDIUM),
      pod("m3.1", LOW, "machine3", MEDIUM), pod("m3.2", LOW, "machine3", MEDIUM)], {"machine3"}),
    ("when highest priorities are the same, minimum sum of priorities is picked", ["machine1", "machine2", "machine3"],
     pod("machine1", HIGH, containers=VLARGE),
     [pod("m1.1", MID, "machine1", MEDIUM), pod("m1.2", MID, "machine1", LARGE),
      pod("m2.1", MID, "machine2", LARGE), pod("m2.2", LOW, "machine2", MEDIUM),
      pod("m3.1", MID, "machine3", MEDIUM), pod("m3.2", MID, "machine3", MEDIUM)], {"machine2"}),
    ("when highest priority and sum are the same, minimum number of pods is picked",
     ["machine1", "machine2", "machine3"], pod("machine1", HIGH, containers=VLARGE),
     [pod("m1.1", MID, "machine1", SMALL), pod("m1.2", NEG, "machine1", SMALL), pod("m1.3", MID, "machine1", SMALL),
      pod("m1.4", NEG, "machine1", SMALL), pod("m2.1", MID, "machine2", LARGE), pod("m2.2", NEG, "machine2", MEDIUM),
      pod("m3.1", MID, "machine3", MEDIUM), pod("m3.2", NEG, "machine3", SMALL), pod("m3.3", LOW, "machine3", SMALL)],
     {"machine2"}),
    ("sum of adjusted priorities is considered", ["machine1", "machine2", "machine3"],
     pod("machine1", HIGH, containers=VLARGE),
     [pod("m1.1", MID, "machine1", SMALL), pod("m1.2", NEG, "machine1", SMALL), pod("m1.3", NEG, "machine1", SMALL),
      pod("m2.1", MID, "machine2", LARGE), pod("m2.2", NEG, "machine2", MEDIUM),
      pod("m3.1", MID, "machine3", MEDIUM), pod("m3.2", NEG, "machine3", SMALL), pod("m3.3", LOW, "machine3", SMALL)],
     {"machine2"}),
    ("non-overlapping lowest high priority, sum priorities, and number of pods",
     ["machine1", "machine2", "machine3", "machine4"], pod("pod1", VHIGH, containers=VLARGE),
     [pod("m1.1", MID, "machine1", SMALL), pod("m1.2", LOW, "machine1", SMALL), pod("m1.3", LOW, "machine1", SMALL),
      pod("m2.1", HIGH, "machine2", LARGE),
      pod("m3.1", MID, "machine3", MEDIUM), pod("m3.2", LOW, "machine3", SMALL), pod("m3.3", LOW, "machine3", SMALL),
      pod("m3.4", LOW, "machine3", MEDIUM),
      pod("m4.1", MID, "machine4", MEDIUM), pod("m4.2", MID, "machine4", SMALL), pod("m4.3", MID, "machine4", SMALL),
      pod("m4.4", NEG, "machine4", SMALL)], {"machine1"}),
]


def test_pick_one_node_for_preemption_table():
    for name, nodes, p, pods, expected in PICK_CASES:
        cache, gs = setup(nodes, pods, [FITS])
        cands = select_nodes_for_preemption(gs, p, PodInfo(p), cache.node_list())
        assert pick_one_node_for_preemption(cands) in expected, name


def test_pick_prefers_fewest_pdb_violations():
    hi, lo = pod("x", MID), pod("y", LOW)
    cands = {"n1": Victims([hi], 1), "n2": Victims([hi, hi, lo], 0)}
    assert pick_one_node_for_preemption(cands) == "n2"
    assert pick_one_node_for_preemption({}) is None


INSUFF_MEM = "Insufficient memory"
SELECTOR = "node(s) didn't match node selector"
HOST = "node(s) didn't match the requested hostname"
TAINTS = "node(s) had taints that the pod didn't tolerate"
LABELS = "node(s) didn't have the requested labels"
AFFINITY = "node(s) didn't match pod affinity rules"
UNSCHED = "node(s) were unschedulable"
OUT_OF_DISK = "node(s) were out of disk space"
DISK = "node(s) had no available disk"

MIGHT_HELP_CASES = [
    ("No node should be attempted", {"machine1": (SELECTOR,), "machine2": (HOST,), "machine3": (TAINTS,),
                                     "machine4": (LABELS,)}, set()),
    ("pod affinity should be tried", {"machine1": (AFFINITY,), "machine2": (HOST,), "machine3": (UNSCHED,)},
     {"machine1", "machine4"}),
    ("pod with both pod affinity and anti-affinity should be tried", {"machine1": (AFFINITY,), "machine2": (HOST,)},
     {"machine1", "machine3", "machine4"}),
    ("Mix of failed predicates works fine", {"machine1": (SELECTOR, OUT_OF_DISK, INSUFF_MEM), "machine2": (HOST, DISK),
                                            "machine3": (INSUFF_MEM,), "machine4": ()}, {"machine3", "machine4"}),
]


def test_nodes_where_preemption_might_help_table():
    nodes = [f"machine{i}" for i in range(1, 5)]
    for name, failed, expected in MIGHT_HELP_CASES:
        assert set(nodes_where_preemption_might_help(pod("pod1", 0), nodes, failed)) == expected, name


class FakeExtender:
    """generic_scheduler_test FakeExtender: filters by a node-name predicate."""

    def __init__(self, ok):
        self.ok = ok
        self.extenders = []

    def filter(self, pod, nodes):
        keep = [n for n in nodes if self.ok(n.name)]
        return keep, {n.name: "extender" for n in nodes if not self.ok(n.name)}

    def prioritize(self, pod, nodes):
        return {}


PREEMPT_FAILED = {"machine1": INSUFF_MEM, "machine2": "node(s) had no available disk", "machine3": INSUFF_MEM}

PREEMPT_CASES = [
    ("basic preemption logic", [pod("m1.1", LOW, "machine1", SMALL), pod("m1.2", LOW, "machine1", SMALL),
                                pod("m2.1", HIGH, "machine2", LARGE), pod("m3.1", MID, "machine3", MEDIUM)],
     None, "machine1", {"m1.1", "m1.2"}),
    ("One node doesn't need any preemption", [pod("m1.1", LOW, "machine1", SMALL), pod("m1.2", LOW, "machine1", SMALL),
                                             pod("m2.1", HIGH, "machine2", LARGE)], None, "machine3", set()),
    ("Scheduler extenders allow only machine1, otherwise machine3 would have been chosen",
     [pod("m1.1", MID, "machine1", SMALL), pod("m1.2", LOW, "machine1", SMALL), pod("m2.1", MID, "machine2", LARGE)],
     [FakeExtender(lambda n: True), FakeExtender(lambda n: n == "machine1")], "machine1", {"m1.1", "m1.2"}),
    ("Scheduler extenders do not allow any preemption",
     [pod("m1.1", MID, "machine1", SMALL), pod("m1.2", LOW, "machine1", SMALL), pod("m2.1", MID, "machine2", LARGE)],
     [FakeExtender(lambda n: False)], None, set()),
]


def test_preempt_table():
    for name, pods, extenders, exp_node, exp_victims in PREEMPT_CASES:
        cache = SchedulerCache()
        for p in pods:            # the reference adds the pods before the nodes
            cache.add_pod(p)
        for n in ("machine1", "machine2", "machine3"):
            cache.add_node(make_node(n))
        gs = GenericScheduler(cache, [FITS], priorities={}, extenders=extenders, equivalence_cache=False)
        p = pod("pod1", HIGH, containers=VLARGE)
        node, victims, _ = preempt(gs, p, PodInfo(p), FitError(p, 3, PREEMPT_FAILED), queue=SchedulingQueue())
        assert node == exp_node, name
        assert names(victims) == exp_victims, name


# -- scheduling_queue_test.go: the nominated-pods half of PriorityQueue --------------------------

def qpod(name, ns, prio, nominated=None, extra=None):
    ann = dict(extra or {})
    if nominated:
        ann[NOMINATED_ANNOTATION] = nominated
    return {"metadata": {"name": name, "namespace": ns, "uid": name + ns, "annotations": ann},
            "spec": {"priority": prio}}


HPP = qpod("hpp", "ns1", HIGH)
HPP_NOM = qpod("hpp", "ns1", HIGH, "node1")
MPP = qpod("mpp", "ns2", (LOW + HIGH) // 2, "node1", {"annot2": "val2"})
UP = qpod("up", "ns1", LOW, "node1", {"annot2": "val2"})


def nominated_names(q):
    return {n: [p["metadata"]["name"] for p in q.waiting_pods_for_node(n)] for n in q.nominated_pods}


def test_queue_add_indexes_and_pop_removes_nominations():
    q = SchedulingQueue()
    for p in (MPP, UP, HPP):
        q.add(p)
    assert nominated_names(q) == {"node1": ["mpp", "up"]}
    assert [q.pop_nowait()[0]["metadata"]["name"] for _ in range(3)] == ["hpp", "mpp", "up"]
    assert q.nominated_pods == {} and q.nominated == {}


def test_queue_add_unschedulable_keeps_nomination():
    q = SchedulingQueue()
    q.add(HPP_NOM)
    q.add_unschedulable(HPP_NOM)        # already active: nothing changes
    q.add(MPP)
    q.add_unschedulable(UP)
    assert nominated_names(q) == {"node1": ["hpp", "mpp", "up"]}
    assert q.pop_nowait()[0] is HPP_NOM and q.pop_nowait()[0] is MPP
    assert nominated_names(q) == {"node1": ["up"]}
    assert "ns1/up" in q.unschedulable


def test_queue_update_and_delete():
    q = SchedulingQueue()
    q.update(None, HPP)
    assert "ns1/hpp" in q.active and q.nominated_pods == {}
    q.update(HPP, HPP_NOM)              # gains a nomination while active
    assert len(q.active) == 1 and nominated_names(q) == {"node1": ["hpp"]}
    q.update(UP, UP)
    q.update(UP, UP)
    assert not q.unschedulable and "ns1/up" in q.active
    assert q.pop_nowait()[0] is HPP_NOM
    q.add(HPP_NOM)
    q.delete(HPP_NOM)
    assert nominated_names(q) == {"node1": ["up"]}
    q.delete(UP)
    assert q.nominated_pods == {}


def test_queue_waiting_pods_for_node_and_clear():
    q = SchedulingQueue()
    for p in (MPP, UP, HPP):
        q.add(p)
    assert q.pop_nowait()[0] is HPP
    assert q.waiting_pods_for_node("node1") == [MPP, UP]
    assert q.waiting_pods_for_node("node2") == []
    cleared = qpod("up", "ns1", LOW, "", {"annot2": "val2"})      # RemoveNominatedNodeAnnotation writes ""
    q.update(UP, cleared)
    assert q.waiting_pods_for_node("node1") == [MPP]
    q.nominate(MPP, "node2")                                        # local nomination ahead of the informer
    assert q.waiting_pods_for_node("node1") == [] and len(q.waiting_pods_for_node("node2")) == 1


def test_queue_assigned_pod_added_moves_affinity_pods():
    aff = qpod("afp", "ns1", 50)
    aff["spec"]["affinity"] = {"podAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [{
        "labelSelector": {"matchExpressions": [{"key": "service", "operator": "In", "values": ["securityscan"]}]},
        "topologyKey": "region"}]}}
    q = SchedulingQueue()
    q.add(MPP)
    q.add_unschedulable(UP)
    q.add_unschedulable(aff)
    q.assigned_pod_added({"metadata": {"name": "lbp", "namespace": "ns1", "labels": {"service": "securityscan"}},
                          "spec": {"nodeName": "machine1"}})
    assert "ns1/afp" in q.active and "ns1/afp" not in q.unschedulable
    assert "ns1/up" in q.unschedulable


# -- MI355X: device-aware nominations --------------------------------------------------------------

def bound_gpu(name, ids, prio, node="n0", labels=None):
    p = gpu_pod(name, len(ids))
    p["spec"]["nodeName"] = node
    p["spec"]["priority"] = prio
    p["spec"]["extendedResources"][0]["assigned"] = list(ids)
    if labels:
        p["metadata"]["labels"] = labels
    return p


def test_nominee_holds_freed_gpus_against_lower_priority_pods():
    """A 4-GPU preemptor nominated to n0 holds the 4 free GPUs there; a lower-priority 1-GPU pod
    created in the victims' grace window must not take them, an equal-priority one may not
    either, a higher-priority one may."""
    cache = SchedulerCache()
    cache.add_node(gpu_node("n0", [gpu_dev(i) for i in range(8)]))
    for i in range(4, 8):
        cache.add_pod(bound_gpu(f"keep{i}", [f"g{i}"], 500))
    q = SchedulingQueue()
    gs = GenericScheduler(cache)
    gs.queue = q
    big = gpu_pod("big", 4, annotations={NOMINATED_ANNOTATION: "n0"})
    big["spec"]["priority"] = 1000
    q.add_unschedulable(big)
    for prio, fits in ((0, False), (1000, False), (2000, True)):
        small = gpu_pod(f"small{prio}", 1)
        small["spec"]["priority"] = prio
        try:
            host, binding = gs.schedule(small, PodInfo(small))
            assert fits, prio
            assert host == "n0" and len(binding["er"]["resources"]) == 1
        except FitError:
            assert not fits, prio
    # the preemptor itself is not its own competitor
    q2 = SchedulingQueue()
    gs.queue = q2
    host, binding = gs.schedule(big, PodInfo(big))
    assert host == "n0" and len(binding["er"]["resources"]) == 4


def test_nominee_reserves_whole_hive_for_xgmi_required():
    """Two hives of 4; the nominee needs a fully connected 4-set and hive h1 is free: a 1-GPU
    pod of lower priority is still placed, but only in the other hive's free GPU."""
    cache = SchedulerCache()
    devs = [gpu_dev(i, hive="h0" if i < 4 else "h1", links="3") for i in range(8)]
    cache.add_node(gpu_node("n0", devs))
    for i in range(3):
        cache.add_pod(bound_gpu(f"h0-{i}", [f"g{i}"], 500))
    q = SchedulingQueue()
    gs = GenericScheduler(cache)
    gs.queue = q
    big = gpu_pod("big", 4, annotations={NOMINATED_ANNOTATION: "n0", "amd.com/xgmi-policy": "required"})
    big["spec"]["priority"] = 1000
    q.add_unschedulable(big)
    small = gpu_pod("small", 1)
    small["spec"]["priority"] = 0
    host, binding = gs.schedule(small, PodInfo(small))
    assert binding["er"]["resources"] == ["g3"]


def test_pdb_violating_victims_are_reprieved_first():
    """With a PDB allowing no disruption over app=db, the victim set avoids db pods when
    non-violating pods of the same priority free enough GPUs."""
    cache = SchedulerCache()
    cache.add_node(gpu_node("n0", [gpu_dev(i) for i in range(4)]))
    cache.add_pod(bound_gpu("db0", ["g0"], 0, labels={"app": "db"}))
    cache.add_pod(bound_gpu("db1", ["g1"], 0, labels={"app": "db"}))
    cache.add_pod(bound_gpu("web0", ["g2"], 0, labels={"app": "web"}))
    cache.add_pod(bound_gpu("web1", ["g3"], 0, labels={"app": "web"}))
    pdb = {"metadata": {"name": "db", "namespace": "default"},
           "spec": {"selector": {"matchLabels": {"app": "db"}}}, "status": {"disruptionsAllowed": 0}}
    gs = GenericScheduler(cache)
    hi = gpu_pod("hi", 2)
    hi["spec"]["priority"] = 100
    victims, n_viol, fits = select_victims_on_node(gs, hi, PodInfo(hi), cache.nodes["n0"], [pdb])
    assert fits and n_viol == 0 and names(victims) == {"web0", "web1"}
    # needing all four GPUs, two PDB violations are unavoidable and are counted
    hi4 = gpu_pod("hi4", 4)
    hi4["spec"]["priority"] = 100
    victims, n_viol, fits = select_victims_on_node(gs, hi4, PodInfo(hi4), cache.nodes["n0"], [pdb])
    assert fits and n_viol == 2 and len(victims) == 4


def test_not_eligible_while_victims_terminate():
    cache = SchedulerCache()
    cache.add_node(gpu_node("n0", [gpu_dev(i) for i in range(2)]))
    v = bound_gpu("v", ["g0"], 0)
    v["metadata"]["deletionTimestamp"] = "2026-01-01T00:00:00Z"
    cache.add_pod(v)
    cache.add_pod(bound_gpu("w", ["g1"], 0))
    hi = gpu_pod("hi", 2, annotations={NOMINATED_ANNOTATION: "n0"})
    hi["spec"]["priority"] = 100
    assert not pod_eligible_to_preempt_others(hi, cache)
    gs = GenericScheduler(cache)
    assert preempt(gs, hi, PodInfo(hi), FitError(hi, 1, {"n0": f"Insufficient {core.AMD_GPU}"})) == (None, [], [])
    # without a nomination (or nominated elsewhere) it may preempt
    fresh = gpu_pod("hi2", 2)
    fresh["spec"]["priority"] = 100
    assert pod_eligible_to_preempt_others(fresh, cache)
    node, victims, _ = preempt(gs, fresh, PodInfo(fresh), FitError(fresh, 1, {"n0": f"Insufficient {core.AMD_GPU}"}))
    assert node == "n0" and names(victims) == {"v", "w"}


def test_unhelpful_nodes_clear_own_nomination():
    cache = SchedulerCache()
    cache.add_node(gpu_node("n0", [gpu_dev(0)]))
    cache.add_pod(bound_gpu("v", ["g0"], 0))
    gs = GenericScheduler(cache)
    hi = gpu_pod("hi", 1, annotations={NOMINATED_ANNOTATION: "n0"})
    hi["spec"]["priority"] = 100
    node, victims, clear = preempt(gs, hi, PodInfo(hi), FitError(hi, 1, {"n0": TAINTS}))
    assert node is None and victims == [] and clear == [hi]


def test_lower_priority_nominees_are_cleared():
    cache = SchedulerCache()
    cache.add_node(gpu_node("n0", [gpu_dev(i) for i in range(2)]))
    cache.add_pod(bound_gpu("v0", ["g0"], 0))
    cache.add_pod(bound_gpu("v1", ["g1"], 0))
    q = SchedulingQueue()
    mid = gpu_pod("mid", 1, annotations={NOMINATED_ANNOTATION: "n0"})
    mid["spec"]["priority"] = 50
    q.add_unschedulable(mid)
    gs = GenericScheduler(cache)
    gs.queue = q
    hi = gpu_pod("hi", 2)
    hi["spec"]["priority"] = 100
    node, victims, clear = preempt(gs, hi, PodInfo(hi), FitError(hi, 1, {"n0": f"Insufficient {core.AMD_GPU}"}), queue=q)
    assert node == "n0" and names(victims) == {"v0", "v1"} and [p["metadata"]["name"] for p in clear] == ["mid"]


# -- end to end: victims with a real termination window ---------------------------------------------

def test_preemption_e2e_grace_window_holds_gpus(run):
    """Victims take their grace period to terminate (two drain in 1 s, two ignore SIGTERM and
    are killed at 6 s). The preemptor preempts exactly once, keeps its NominatedNodeName
    annotation, and a lower-priority 1-GPU pod created during the window never gets the GPUs
    freed for it."""
    import asyncio
    from kubernetes_amd.cluster import LocalCluster
    from kubernetes_amd.kubelet.runtime.stub import STOP_SECONDS

    async def main():
        async with LocalCluster(nodes=1, gpus_per_node=8) as cl:
            c = cl.client
            for name, value in (("high", 1000), ("mid", 10), ("five", 5)):
                await c.create("priorityclasses", {"apiVersion": "scheduling.k8s.io/v1alpha1", "kind": "PriorityClass",
                                                   "metadata": {"name": name}, "value": value})

            def gpu(n):
                return [{"name": "c", "image": "x", "resources": {"limits": {core.AMD_GPU: str(n)}}}]
            for i in range(8):
                spec = {"containers": gpu(1), "terminationGracePeriodSeconds": 6}
                if i < 4:
                    spec["priorityClassName"] = "mid"
                ann = {STOP_SECONDS: "1" if i in (4, 5) else "30"}
                await c.create("pods", {"metadata": {"name": f"low{i}", "annotations": ann}, "spec": spec})
            for i in range(8):
                await cl.wait_pod(f"low{i}")
            await c.create("pods", {"metadata": {"name": "big"}, "spec": {"priorityClassName": "high",
                                                                           "containers": gpu(4)}})
            node = cl.nodes[0].name

            async def nominated():
                p = await c.get("pods", "big", "default")
                return (p["metadata"].get("annotations") or {}).get(NOMINATED_ANNOTATION) == node
            await cl.wait_for(nominated, timeout=15)
            terminating = [p["metadata"]["name"] for p in (await c.list("pods", "default"))["items"]
                           if p["metadata"].get("deletionTimestamp")]
            assert sorted(terminating) == ["low4", "low5", "low6", "low7"]
            await c.create("pods", {"metadata": {"name": "sneak"}, "spec": {"priorityClassName": "five",
                                                                             "containers": gpu(1)}})
            # the two fast victims are gone after ~1 s: 2 GPUs are free, but reserved for "big"
            async def fast_gone():
                names = {p["metadata"]["name"] for p in (await c.list("pods", "default"))["items"]}
                return "low4" not in names and "low5" not in names
            await cl.wait_for(fast_gone, timeout=10)
            await asyncio.sleep(1.0)
            sneak = await c.get("pods", "sneak", "default")
            assert not sneak["spec"].get("nodeName"), "the lower-priority pod took GPUs freed for the preemptor"
            big = await cl.wait_pod("big", timeout=20)
            assert len(big["spec"]["extendedResources"][0]["assigned"]) == 4
            assert (big["metadata"].get("annotations") or {}).get(NOMINATED_ANNOTATION) == node
            assert cl.scheduler.m_preemptions.value() == 1
            sneak = await c.get("pods", "sneak", "default")
            assert not sneak["spec"].get("nodeName")
            ev = [e for e in (await c.list("events", "default"))["items"] if e.get("reason") == "Preempted"]
            assert sorted(e["involvedObject"]["name"] for e in ev) == ["low4", "low5", "low6", "low7"]
    run(main(), timeout=120)
