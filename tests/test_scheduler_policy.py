"""Scheduler Policy parity: every name the reference's algorithm provider registers that a Policy
file can use, the argument-based custom predicates / priorities, and the reference's own example
policies.

Parity:
  * `plugin/pkg/scheduler/algorithmprovider/defaults/defaults.go:67-162` — `PodFitsPorts`
    (deprecated alias of PodFitsHostPorts), `GeneralPredicates`, `ServiceSpreadingPriority`,
    `EqualPriority`;
  * `plugin/pkg/scheduler/factory/plugins.go:198-340` + `api/types.go:75-120` —
    `predicates[].argument.{serviceAffinity{labels}, labelsPresence{labels,presence}}`,
    `priorities[].argument.{serviceAntiAffinity{label}, labelPreference{label,presence}}`;
  * `predicates/predicates_test.go` TestServiceAffinity / TestNodeLabelPresence,
    `priorities/selector_spreading_test.go` TestZoneSpreadPriority (ServiceAntiAffinity),
    `priorities/node_label_test.go`, `factory/factory_test.go` TestCreateFromConfig
    (the example policies load);
  * `examples/scheduler-policy-config.json`, `examples/scheduler-policy-config-with-extender.json`.
"""
import json
import os

import pytest

from kubernetes_amd.scheduler import policy as SP
from kubernetes_amd.scheduler import predicates as P
from kubernetes_amd.scheduler import priorities as PR
from kubernetes_amd.scheduler.cache import PodInfo, SchedulerCache
from kubernetes_amd.scheduler.generic import CycleContext, FitError, GenericScheduler

REF_EXAMPLES = "/root/reference/examples"
HERE = os.path.dirname(os.path.abspath(__file__))


def node(name, labels=None, cpu="8", pods="110"):
    return {"metadata": {"name": name, "labels": labels or {}}, "spec": {},
            "status": {"allocatable": {"cpu": cpu, "memory": "64Gi", "pods": pods},
                       "conditions": [{"type": "Ready", "status": "True"}]}}


def pod(name, labels=None, node_name=None, ns="default", selector=None, ports=None, cpu=None):
    c = {"name": "c", "image": "x"}
    if ports:
        c["ports"] = [{"containerPort": p, "hostPort": p} for p in ports]
    if cpu:
        c["resources"] = {"requests": {"cpu": cpu}}
    p = {"metadata": {"name": name, "namespace": ns, "uid": "u-" + name, "labels": labels or {}},
         "spec": {"containers": [c]}}
    if node_name:
        p["spec"]["nodeName"] = node_name
    if selector:
        p["spec"]["nodeSelector"] = selector
    return p


def svc(name, selector, ns="default"):
    return {"metadata": {"name": name, "namespace": ns}, "spec": {"selector": selector}}


def cluster(nodes, pods=(), services=()):
    c = SchedulerCache()
    for n in nodes:
        c.add_node(n)
    for p in pods:
        c.add_pod(p)
    for s in services:
        c.set_service(s)
    return c


def _ctx(cache, p):
    return CycleContext(cache, p)


def _fits(fn, cache, p, node_name):
    return fn(p, PodInfo(p), cache.nodes[node_name], _ctx(cache, p))


# -- example policies ------------------------------------------------------------------------
@pytest.mark.parametrize("fname", ["scheduler-policy-config.json", "scheduler-policy-config-with-extender.json"])
def test_reference_example_policies_load(fname):
    path = os.path.join(REF_EXAMPLES, fname)
    if not os.path.exists(path):
        pytest.skip("reference examples not present")
    with open(path) as f:
        algo = SP.parse_policy(f.read())
    preds, prios, ext = algo
    assert "PodFitsHostPorts" in preds and "HostName" in preds
    assert prios["ServiceSpreadingPriority"] == 1 and prios["EqualPriority"] == 1
    assert algo.hard_pod_affinity_symmetric_weight == 10
    if "extender" in fname:
        assert ext[0]["urlPrefix"] == "http://127.0.0.1:12346/scheduler" and ext[0]["weight"] == 5
    # and the algorithm builds and schedules with it
    cache = cluster([node("a"), node("b")])
    gs = GenericScheduler(cache, preds, prios)
    assert gs.schedule(pod("p"))[0] in ("a", "b")


def test_extender_policy_round_trips_through_the_scheduler_cmd_loader(tmp_path, run):
    pol = {"kind": "Policy", "apiVersion": "v1",
           "predicates": [{"name": "PodFitsPorts"}, {"name": "GeneralPredicates"}],
           "priorities": [{"name": "EqualPriority", "weight": 2}],
           "extenders": [{"urlPrefix": "http://127.0.0.1:1/sched", "filterVerb": "filter", "prioritizeVerb": "prio",
                          "weight": 3, "enableHttps": False, "nodeCacheCapable": True}],
           "hardPodAffinitySymmetricWeight": 7}
    f = tmp_path / "policy.json"
    f.write_text(json.dumps(pol))

    async def main():
        return await SP.resolve_algorithm(None, policy_file=str(f))
    algo = run(main())
    preds, prios, ext = algo
    assert preds == ["PodFitsPorts", "GeneralPredicates"] and prios == {"EqualPriority": 2}
    assert ext == pol["extenders"] and algo.hard_pod_affinity_symmetric_weight == 7
    from kubernetes_amd.scheduler.extender import HTTPExtender
    e = HTTPExtender.from_config(ext[0])
    assert e is not None


def test_policy_validation_errors():
    bad = [
        {"predicates": [{"name": "X", "argument": {}}]},                                    # no argument kind
        {"predicates": [{"name": "X", "argument": {"serviceAffinity": {"labels": ["a"]},
                                                   "labelsPresence": {"labels": ["a"]}}}]},   # two kinds
        {"priorities": [{"name": "Y", "weight": 1, "argument": {"labelPreference": {}}}]},  # no label
        {"priorities": [{"name": "Y", "weight": 0, "argument": {"labelPreference": {"label": "a"}}}]},
        {"hardPodAffinitySymmetricWeight": 101},
        {"extenders": [{"filterVerb": "f"}]},
    ]
    for pol in bad:
        with pytest.raises(SP.PolicyError):
            SP.parse_policy(json.dumps({"kind": "Policy", **pol}))


# -- registry names ---------------------------------------------------------------------------
def test_pod_fits_ports_is_the_host_ports_predicate():
    cache = cluster([node("a")], [pod("x", node_name="a", ports=[8080])])
    assert _fits(P.PREDICATES["PodFitsPorts"], cache, pod("p", ports=[8080]), "a")
    assert _fits(P.PREDICATES["PodFitsPorts"], cache, pod("q", ports=[9090]), "a") is None


def test_general_predicates():
    cache = cluster([node("a", {"zone": "z1"}, cpu="1"), node("b", {"zone": "z2"})],
                    [pod("x", node_name="b", ports=[80])])
    gp = P.PREDICATES["GeneralPredicates"]
    assert "Insufficient cpu" in _fits(gp, cache, pod("p", cpu="2"), "a")              # resources
    assert "ports" in _fits(gp, cache, pod("p", ports=[80]), "b")                       # host ports
    assert "node selector" in _fits(gp, cache, pod("p", selector={"zone": "z1"}), "b")  # selector
    p = pod("p")
    p["spec"]["nodeName"] = "a"
    assert "hostname" in _fits(gp, cache, p, "b")                                       # host
    assert _fits(gp, cache, pod("p", selector={"zone": "z2"}), "b") is None


def test_equal_priority_and_service_spreading():
    cache = cluster([node("a"), node("b"), node("c")],
                    [pod("w1", {"app": "web"}, "a"), pod("w2", {"app": "web"}, "a"), pod("w3", {"app": "web"}, "b"),
                     pod("o1", {"app": "other"}, "c"), pod("w4", {"app": "web"}, "c", ns="elsewhere")],
                    [svc("web", {"app": "web"})])
    gs = GenericScheduler(cache, ["PodFitsResources"], {"ServiceSpreadingPriority": 1})
    p = pod("new", {"app": "web"})
    ctx = _ctx(cache, p)
    scores = gs.prioritize(p, PodInfo(p), cache.node_list(), ctx)
    # counts a=2, b=1, c=0 (other app / other namespace do not count) -> 10*(2-n)/2
    assert scores == {"a": 0.0, "b": 5.0, "c": 10.0}
    assert gs.schedule(p)[0] == "c"
    gs = GenericScheduler(cache, ["PodFitsResources"], {"EqualPriority": 3})
    assert set(gs.prioritize(p, PodInfo(p), cache.node_list(), ctx).values()) == {3.0}
    # a pod no service selects: ServiceSpreading does not apply
    assert gs.schedule(pod("lonely", {"app": "none"}))[0] in ("a", "b", "c")


def test_selector_spread_counts_service_siblings():
    cache = cluster([node("a"), node("b")], [pod("w1", {"app": "web"}, "a")], [svc("web", {"app": "web"})])
    gs = GenericScheduler(cache, ["PodFitsResources"], {"SelectorSpreadPriority": 1})
    assert gs.schedule(pod("new", {"app": "web"}))[0] == "b"


# -- argument-based predicates ---------------------------------------------------------------
def test_labels_presence_table():
    n_with = node("with", {"gpu": "mi355x", "rack": "r1"})
    n_without = node("without", {"rack": "r2"})
    cache = cluster([n_with, n_without])
    cases = [  # labels, presence, node, fits
        (["gpu"], True, "with", True), (["gpu"], True, "without", False),
        (["gpu"], False, "with", False), (["gpu"], False, "without", True),
        (["gpu", "rack"], True, "with", True), (["gpu", "rack"], True, "without", False),
        (["gpu", "rack"], False, "without", False), (["foo"], False, "with", True),
    ]
    for labels, presence, n, fits in cases:
        fn = P.make_labels_presence(labels, presence)
        got = _fits(fn, cache, pod("p"), n)
        assert (got is None) == fits, (labels, presence, n, got)


def test_service_affinity_table():
    """`predicates_test.go` TestServiceAffinity shapes: the first placed pod of the service pins
    the label values; the pod's own nodeSelector wins; no service -> anything fits."""
    nodes = [node("m1", {"region": "r1", "zone": "z11"}), node("m2", {"region": "r1", "zone": "z12"}),
             node("m3", {"region": "r2", "zone": "z21"})]
    labels = ["region"]
    fn = P.make_service_affinity(labels)
    # no pods yet, service exists: the first pod may go anywhere
    cache = cluster(nodes, [], [svc("s", {"app": "a"})])
    assert all(_fits(fn, cache, pod("p", {"app": "a"}), n) is None for n in ("m1", "m2", "m3"))
    # a service-mate on m1 (region r1): m2 fits (same region), m3 does not
    cache = cluster(nodes, [pod("q", {"app": "a"}, "m1")], [svc("s", {"app": "a"})])
    assert _fits(fn, cache, pod("p", {"app": "a"}), "m2") is None
    assert "service affinity" in _fits(fn, cache, pod("p", {"app": "a"}), "m3")
    # the pod's own nodeSelector supplies the region: r2 only, whatever its mates do
    assert _fits(fn, cache, pod("p", {"app": "a"}, selector={"region": "r2"}), "m3") is None
    assert _fits(fn, cache, pod("p", {"app": "a"}, selector={"region": "r2"}), "m1")
    # no service selects the pod: no constraint from the mates
    cache = cluster(nodes, [pod("q", {"app": "a"}, "m1")], [])
    assert _fits(fn, cache, pod("p", {"app": "a"}), "m3") is None
    # two labels: region and zone both pinned by the mate
    fn2 = P.make_service_affinity(["region", "zone"])
    cache = cluster(nodes, [pod("q", {"app": "a"}, "m1")], [svc("s", {"app": "a"})])
    assert _fits(fn2, cache, pod("p", {"app": "a"}), "m1") is None
    assert _fits(fn2, cache, pod("p", {"app": "a"}), "m2")
    # a mate in another namespace does not count
    cache = cluster(nodes, [pod("q", {"app": "a"}, "m1", ns="other")], [svc("s", {"app": "a"})])
    assert _fits(fn, cache, pod("p", {"app": "a"}), "m3") is None


def test_service_affinity_policy_end_to_end():
    algo = SP.parse_policy(json.dumps({
        "kind": "Policy",
        "predicates": [{"name": "PodFitsResources"},
                       {"name": "RegionAffinity", "argument": {"serviceAffinity": {"labels": ["region"]}}},
                       {"name": "RequireGPU", "argument": {"labelsPresence": {"labels": ["gpu"], "presence": True}}}],
        "priorities": [{"name": "EqualPriority", "weight": 1}]}))
    preds, prios, _ = algo
    nodes = [node("m1", {"region": "r1", "gpu": "y"}), node("m2", {"region": "r1"}), node("m3", {"region": "r2", "gpu": "y"})]
    cache = cluster(nodes, [pod("q", {"app": "a"}, "m1")], [svc("s", {"app": "a"})])
    gs = GenericScheduler(cache, preds, prios)
    assert not gs.use_ecache or gs.global_view          # global-view plugin: no equivalence cache reuse
    assert gs.schedule(pod("p", {"app": "a"}))[0] == "m1"   # m2 lacks gpu, m3 is in another region
    with pytest.raises(FitError) as e:
        gs.schedule(pod("p2", {"app": "a"}, selector={"region": "r3"}))
    assert "service affinity" in str(e.value)


# -- argument-based priorities ---------------------------------------------------------------
def test_label_preference_table():
    cache = cluster([node("a", {"ssd": "true"}), node("b")])
    for presence, want in ((True, {"a": 10.0, "b": 0.0}), (False, {"a": 0.0, "b": 10.0})):
        fn = PR.make_label_preference("ssd", presence)
        p = pod("p")
        got = {n: fn(p, PodInfo(p), cache.nodes[n], _ctx(cache, p)) for n in ("a", "b")}
        assert got == want


def test_service_anti_affinity_table():
    """`selector_spreading_test.go` TestZoneSpreadPriority shape: zone z1 holds 2 of the
    service's 4 pods, z2 holds 1, one sits on an unlabeled node; unlabeled nodes score 0."""
    nodes = [node("a1", {"zone": "z1"}), node("a2", {"zone": "z1"}), node("b1", {"zone": "z2"}),
             node("c1", {"zone": "z3"}), node("x", {})]
    pods = [pod("s1", {"app": "a"}, "a1"), pod("s2", {"app": "a"}, "a2"), pod("s3", {"app": "a"}, "b1"),
            pod("s4", {"app": "a"}, "x"), pod("o", {"app": "b"}, "c1")]
    cache = cluster(nodes, pods, [svc("s", {"app": "a"})])
    fn = PR.make_service_anti_affinity("zone")
    p = pod("new", {"app": "a"})
    ctx = _ctx(cache, p)
    got = {n: fn(p, PodInfo(p), cache.nodes[n], ctx) for n in ("a1", "a2", "b1", "c1", "x")}
    assert got == {"a1": 5.0, "a2": 5.0, "b1": 7.0, "c1": 10.0, "x": 0.0}
    # no service pods yet: every labeled node scores 10
    cache = cluster(nodes, [], [svc("s", {"app": "a"})])
    ctx = _ctx(cache, p)
    assert {n: fn(p, PodInfo(p), cache.nodes[n], ctx) for n in ("a1", "x")} == {"a1": 10.0, "x": 0.0}
    # through a Policy: the pod goes to the emptiest zone
    algo = SP.parse_policy(json.dumps({
        "kind": "Policy", "predicates": [{"name": "PodFitsResources"}],
        "priorities": [{"name": "ZoneSpread", "weight": 2, "argument": {"serviceAntiAffinity": {"label": "zone"}}},
                       {"name": "PreferSSD", "weight": 1, "argument": {"labelPreference": {"label": "ssd", "presence": True}}}]}))
    preds, prios, _ = algo
    cache = cluster(nodes, pods, [svc("s", {"app": "a"})])
    assert GenericScheduler(cache, preds, prios).schedule(pod("n2", {"app": "a"}))[0] == "c1"


def test_policy_via_scheduler_process(run, tmp_path):
    """A policy file with argument-based plugins drives the real scheduler process loop: the
    ServiceAffinity predicate keeps a service's second pod in the first one's region."""
    import asyncio
    from kubernetes_amd.apiserver.server import APIServer
    from kubernetes_amd.client.rest import Client
    from kubernetes_amd.scheduler.scheduler import Scheduler

    async def main():
        api = APIServer()
        port = await api.start()
        c = Client(f"http://127.0.0.1:{port}")
        sched = None
        try:
            for n in (node("m1", {"region": "r1"}), node("m2", {"region": "r2"}), node("m3", {"region": "r2"})):
                n["kind"], n["apiVersion"] = "Node", "v1"
                await c.create("nodes", n)
            await c.create("services", {"kind": "Service", "apiVersion": "v1", "metadata": {"name": "web"},
                                        "spec": {"selector": {"app": "web"}, "ports": [{"port": 80}]}}, "default")
            preds, prios, _ = SP.parse_policy(json.dumps({
                "kind": "Policy",
                "predicates": [{"name": "GeneralPredicates"},
                               {"name": "Region", "argument": {"serviceAffinity": {"labels": ["region"]}}}],
                "priorities": [{"name": "EqualPriority", "weight": 1}]}))
            sched = Scheduler(c, predicates=preds, priorities=prios, emit_events=False)
            asyncio.ensure_future(sched.run())
            first = pod("w0", {"app": "web"})
            first["kind"], first["apiVersion"] = "Pod", "v1"
            await c.create("pods", first, "default")

            async def node_of(name):
                for _ in range(200):
                    p = await c.get("pods", name, "default")
                    if (p.get("spec") or {}).get("nodeName"):
                        return p["spec"]["nodeName"]
                    await asyncio.sleep(0.02)
                raise AssertionError(f"{name} not scheduled")
            n0 = await node_of("w0")
            region = {"m1": "r1", "m2": "r2", "m3": "r2"}
            for i in range(1, 5):
                p = pod(f"w{i}", {"app": "web"})
                p["kind"], p["apiVersion"] = "Pod", "v1"
                await c.create("pods", p, "default")
                assert region[await node_of(f"w{i}")] == region[n0]
        finally:
            if sched is not None:
                await sched.stop()
            await c.close()
            await api.stop()
    run(main(), timeout=60)
