"""Ported extender tables and extender bind delegation.

Reference: `plugin/pkg/scheduler/core/extender_test.go` TestGenericSchedulerWithExtenders
(:186-330) — fake extenders built from per-node predicates and prioritizers; a filter error
fails scheduling, a prioritize error is ignored, extender scores are multiplied by the
extender's weight and added to the scheduler's own. `core/extender.go:198` Bind /
`factory.go:886` getBinder and `api/validation/validation.go:37` (at most one binder) are the
bind-delegation cases; the GPU case checks the device binding reaches the binder extender.
"""
import json

import pytest

from kubernetes_amd.api import core
from kubernetes_amd.cluster import LocalCluster
from kubernetes_amd.scheduler.cache import SchedulerCache
from kubernetes_amd.scheduler.extender import ExtenderError, HTTPExtender
from kubernetes_amd.scheduler.generic import FitError, GenericScheduler
from kubernetes_amd.scheduler.policy import PolicyError, parse_policy
from kubernetes_amd.utils.httpserver import HTTPServer, Response


def error_pred(node):
    raise ExtenderError("Some error")


def false_pred(node):
    return False


def true_pred(node):
    return True


def machine1_pred(node):
    return node == "machine1"


def machine2_pred(node):
    return node == "machine2"


def error_prio(nodes):
    raise ExtenderError("Some error")


def machine1_prio(nodes):
    return {n: 10 if n == "machine1" else 1 for n in nodes}


def machine2_prio(nodes):
    return {n: 10 if n == "machine2" else 1 for n in nodes}


class FakeExtender:
    """extender_test.go:106 FakeExtender: per-node predicates, weighted prioritizers."""

    def __init__(self, predicates=(), prioritizers=(), weight=1):
        self.predicates, self.prioritizers, self.weight = predicates, prioritizers, weight

    def filter(self, pod, nodes):
        keep, failed = [], {}
        for ni in nodes:
            if all(p(ni.name) for p in self.predicates):
                keep.append(ni)
            else:
                failed[ni.name] = "FakeExtender failed"
        return keep, failed

    def prioritize(self, pod, nodes):
        scores = {ni.name: 0 for ni in nodes}
        for fn, w in self.prioritizers:
            for name, s in fn([ni.name for ni in nodes]).items():
                scores[name] += s * w
        return {name: s * self.weight for name, s in scores.items()}


def machine2_priority(pod, pi, ni, ctx):
    return 10 if ni.name == "machine2" else 1


TRUE = [("true", lambda pod, pi, ni, ctx: None)]
EQUAL = {"EqualPriority": 1}

CASES = [
    ("test 1", EQUAL, [FakeExtender([true_pred]), FakeExtender([error_pred])], ["machine1", "machine2"], None),
    ("test 2", EQUAL, [FakeExtender([true_pred]), FakeExtender([false_pred])], ["machine1", "machine2"], None),
    ("test 3", EQUAL, [FakeExtender([true_pred]), FakeExtender([machine1_pred])], ["machine1", "machine2"],
     "machine1"),
    ("test 4", EQUAL, [FakeExtender([machine2_pred]), FakeExtender([machine1_pred])], ["machine1", "machine2"],
     None),
    ("test 5", EQUAL, [FakeExtender([true_pred], [(error_prio, 10)], 1)], ["machine1"], "machine1"),
    ("test 6", EQUAL, [FakeExtender([true_pred], [(machine1_prio, 10)], 1),
                       FakeExtender([true_pred], [(machine2_prio, 10)], 5)], ["machine1", "machine2"], "machine2"),
    # machine2 has higher score: the scheduler's own priority (weight 20) beats the extender's
    ("test 7", {"machine2": (20, machine2_priority, False, None)},
     [FakeExtender([true_pred], [(machine1_prio, 10)], 1)], ["machine1", "machine2"], "machine2"),
]


def _node(name):
    return {"metadata": {"name": name}, "spec": {},
            "status": {"allocatable": {"cpu": "4", "memory": "8Gi", "pods": "110"},
                       "conditions": [{"type": "Ready", "status": "True"}]}}


@pytest.mark.parametrize("name,prios,extenders,nodes,expected", CASES, ids=[c[0] for c in CASES])
def test_generic_scheduler_with_extenders(name, prios, extenders, nodes, expected):
    cache = SchedulerCache()
    for n in nodes:
        cache.add_node(_node(n))
    gs = GenericScheduler(cache, TRUE, prios, extenders=extenders, equivalence_cache=False)
    pod = {"metadata": {"name": "ignored", "namespace": "default"}, "spec": {"containers": [{"name": "c"}]}}
    if expected is None:
        with pytest.raises((FitError, ExtenderError)):
            gs.schedule(pod)
    else:
        host, _ = gs.schedule(pod)
        assert host == expected, name


def test_prioritize_error_is_ignored_with_several_nodes():
    """generic_scheduler.go PrioritizeNodes: a failing extender leaves the other scores."""
    cache = SchedulerCache()
    for n in ("machine1", "machine2"):
        cache.add_node(_node(n))
    exts = [FakeExtender([true_pred], [(error_prio, 10)], 1), FakeExtender([true_pred], [(machine2_prio, 1)], 3)]
    gs = GenericScheduler(cache, TRUE, EQUAL, extenders=exts, equivalence_cache=False)
    host, _ = gs.schedule({"metadata": {"name": "p", "namespace": "default"}, "spec": {"containers": [{"name": "c"}]}})
    assert host == "machine2"


def test_policy_allows_one_binder():
    ext = {"urlPrefix": "http://127.0.0.1:1/x", "filterVerb": "filter"}
    parse_policy(json.dumps({"kind": "Policy", "extenders": [dict(ext, bindVerb="bind"), ext]}))
    with pytest.raises(PolicyError, match="Only one extender can implement bind, found 2"):
        parse_policy(json.dumps({"kind": "Policy", "extenders": [dict(ext, bindVerb="bind"),
                                                                 dict(ext, BindVerb="bind")]}))
    assert HTTPExtender.from_config(dict(ext, BindVerb="b")).is_binder()
    assert not HTTPExtender.from_config(ext).is_binder()
    with pytest.raises(ExtenderError, match="empty bindVerb"):
        HTTPExtender.from_config(ext).bind("default", "p", "u", "n0")


def test_binder_extender_writes_the_binding(run):
    """A binder extender receives ExtenderBindingArgs (with the device IDs) and binds itself;
    an error result is a rejected binding and the pod is retried."""
    seen = []
    state = {"cluster": None, "fail_first": True}

    async def handler(req):
        args = json.loads(req.body)
        seen.append(args)
        if state["fail_first"]:
            state["fail_first"] = False
            return Response(200, json.dumps({"Error": "not yet"}).encode())
        await state["cluster"].client.bind(args["PodNamespace"], args["PodName"], args["Node"],
                                           args.get("ExtendedResourceBindings"))
        return Response(200, b"{}")

    async def main():
        srv = HTTPServer(handler)
        port = await srv.start()
        try:
            ext = HTTPExtender(f"http://127.0.0.1:{port}/ext", bind_verb="bind")
            async with LocalCluster(nodes=1, gpus_per_node=8, scheduler_kwargs={"extenders": [ext]}) as cl:
                state["cluster"] = cl
                await cl.client.create("pods", {"metadata": {"name": "g"}, "spec": {"containers": [{
                    "name": "c", "image": "x", "resources": {"limits": {core.AMD_GPU: "2"}}}]}})
                p = await cl.wait_pod("g", timeout=30)
                assert len(p["spec"]["extendedResources"][0]["assigned"]) == 2
                assert len(seen) == 2
                args = seen[-1]
                assert args["PodName"] == "g" and args["PodNamespace"] == "default"
                assert args["PodUID"] == p["metadata"]["uid"] and args["Node"] == p["spec"]["nodeName"]
                ids = next(iter(args["ExtendedResourceBindings"].values()))["resources"]
                assert sorted(ids) == sorted(p["spec"]["extendedResources"][0]["assigned"])
                assert cl.scheduler.binder is ext
        finally:
            await srv.stop()
    run(main(), timeout=120)

