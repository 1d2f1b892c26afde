"""DefaultTolerationSeconds — port of
`plugin/pkg/admission/defaulttolerationseconds/admission_test.go` (TestForgivenessAdmission)."""
import pytest

from kubernetes_amd.apiserver.admission import CREATE, Attributes, new_chain

NR, UR = "node.kubernetes.io/not-ready", "node.kubernetes.io/unreachable"
ALPHA_NR, ALPHA_UR = "node.alpha.kubernetes.io/notReady", "node.alpha.kubernetes.io/unreachable"


def t(key=None, effect="NoExecute", seconds=300, op="Exists"):
    out = {"operator": op}
    if key:
        out["key"] = key
    if effect:
        out["effect"] = effect
    if seconds is not None:
        out["tolerationSeconds"] = seconds
    return out


CASES = [
    ("no tolerations", [], [t(NR), t(UR)]),
    ("alpha tolerations are not touched", [t(ALPHA_NR), t(ALPHA_UR)], [t(ALPHA_NR), t(ALPHA_UR), t(NR), t(UR)]),
    ("alpha not-ready", [t(ALPHA_NR)], [t(ALPHA_NR), t(NR), t(UR)]),
    ("alpha unreachable", [t(ALPHA_UR)], [t(ALPHA_UR), t(NR), t(UR)]),
    ("unrelated tolerations", [t("foo", "NoSchedule", None, "Equal") | {"value": "bar"}],
     [t("foo", "NoSchedule", None, "Equal") | {"value": "bar"}, t(NR), t(UR)]),
    ("not-ready specified", [t(NR, seconds=700)], [t(NR, seconds=700), t(UR)]),
    ("unreachable specified", [t(UR, seconds=700)], [t(UR, seconds=700), t(NR)]),
    ("both specified", [t(NR, seconds=700), t(UR, seconds=60)], [t(NR, seconds=700), t(UR, seconds=60)]),
    ("unreachable with empty effect", [t(UR, None, 700)], [t(UR, None, 700), t(NR)]),
    ("wildcard toleration", [t(None, None, 700)], [t(None, None, 700)]),
    # MI355X addition: a NoSchedule-only not-ready toleration does not cover NoExecute
    ("not-ready NoSchedule only", [t(NR, "NoSchedule", None)], [t(NR, "NoSchedule", None), t(NR), t(UR)]),
]


@pytest.mark.parametrize("name,given,want", CASES, ids=[c[0] for c in CASES])
def test_forgiveness_admission(name, given, want):
    pod = {"metadata": {"name": "p", "namespace": "foo"}, "spec": {"tolerations": [dict(x) for x in given]}}
    new_chain(["DefaultTolerationSeconds"]).admit(Attributes(CREATE, "pods", "", "foo", "p", pod))
    assert pod["spec"]["tolerations"] == want


def test_configured_seconds_and_subresources():
    chain = new_chain(["DefaultTolerationSeconds"], None, {"DefaultTolerationSeconds": {
        "defaultNotReadyTolerationSeconds": 60, "defaultUnreachableTolerationSeconds": 90}})
    pod = {"metadata": {"name": "p"}, "spec": {}}
    chain.admit(Attributes(CREATE, "pods", "", "foo", "p", pod))
    assert [x["tolerationSeconds"] for x in pod["spec"]["tolerations"]] == [60, 90]
    other = {"metadata": {"name": "p"}, "spec": {}}
    chain.admit(Attributes(CREATE, "pods", "binding", "foo", "p", other))
    assert other == {"metadata": {"name": "p"}, "spec": {}}


def test_always_pull_images_admit_and_validate():
    """`alwayspullimages/admission_test.go`: TestAdmission sets Always on every container and
    init container; TestValidate refuses any other policy; subresources are ignored."""
    import pytest as _pt
    from kubernetes_amd.apiserver.admission import AdmissionError, UPDATE
    chain = new_chain(["AlwaysPullImages"])
    pod = {"metadata": {"name": "p"}, "spec": {
        "initContainers": [{"name": "i1"}, {"name": "i2", "imagePullPolicy": "IfNotPresent"}],
        "containers": [{"name": "c1", "imagePullPolicy": "Never"}, {"name": "c2", "imagePullPolicy": "Always"}]}}
    a = Attributes(CREATE, "pods", "", "ns", "p", pod)
    chain.admit(a)
    chain.validate(a)
    assert all(c["imagePullPolicy"] == "Always" for k in ("initContainers", "containers") for c in pod["spec"][k])
    bad = {"metadata": {"name": "p"}, "spec": {"containers": [{"name": "c", "imagePullPolicy": "Never"}]}}
    with _pt.raises(AdmissionError, match=r"spec.containers\[0\].imagePullPolicy: Unsupported value: \"Never\""):
        chain.validate(Attributes(UPDATE, "pods", "", "ns", "p", bad, bad))
    chain.validate(Attributes(UPDATE, "pods", "status", "ns", "p", bad, bad))


# -- ExtendedResourceToleration: `plugin/pkg/admission/extendedresourcetoleration/admission_test.go`

ER1, ER2 = "example.com/device-ek", "example.com/device-do"


CPU_C = {"name": "c", "image": "x", "resources": {"requests": {"cpu": "2"}}}
MEM_C = {"name": "m", "image": "x", "resources": {"requests": {"memory": "2048"}}}
ER1_C = {"name": "e1", "image": "x", "resources": {"requests": {ER1: "1"}}}
ER2_C = {"name": "e2", "image": "x", "resources": {"requests": {ER2: "2"}}}
ER1_TOL = {"key": ER1, "operator": "Exists", "effect": "NoSchedule"}
ER2_TOL = {"key": ER2, "operator": "Exists", "effect": "NoSchedule"}
FOO_TOL = {"key": "foo", "operator": "Equal", "value": "bar", "effect": "NoSchedule"}

ERT_CASES = [
    ("empty pod without any extended resources", {}, None),
    ("container without any extended resources", {"containers": [CPU_C]}, None),
    ("init container without any extended resources", {"containers": [CPU_C], "initContainers": [MEM_C]}, None),
    ("container with extended resource", {"containers": [CPU_C, ER1_C]}, [ER1_TOL]),
    ("init container with extended resource", {"containers": [CPU_C], "initContainers": [ER2_C]}, [ER2_TOL]),
    ("existing tolerations preserved", {"containers": [ER1_C], "tolerations": [FOO_TOL]}, [FOO_TOL, ER1_TOL]),
    ("multiple extended resources, sorted", {"containers": [ER1_C, CPU_C], "initContainers": [ER2_C, MEM_C]},
     [ER2_TOL, ER1_TOL]),
    ("existing correct toleration: no change", {"containers": [ER1_C], "tolerations": [ER1_TOL]}, [ER1_TOL]),
    ("same key, different effect and value: both kept",
     {"containers": [ER1_C], "tolerations": [{"key": ER1, "operator": "Equal", "value": "foo", "effect": "NoExecute"}]},
     [{"key": ER1, "operator": "Equal", "value": "foo", "effect": "NoExecute"}, ER1_TOL]),
    ("wildcard toleration preserved", {"containers": [ER1_C], "tolerations": [{"operator": "Exists"}]},
     [{"operator": "Exists"}, ER1_TOL]),
]


@pytest.mark.parametrize("name,spec,want", ERT_CASES, ids=[c[0] for c in ERT_CASES])
def test_extended_resource_toleration(name, spec, want):
    import copy
    chain = new_chain(["ExtendedResourceToleration"])
    pod = {"metadata": {"name": "p", "namespace": "default"}, "spec": copy.deepcopy(spec)}
    chain.admit(Attributes(CREATE, "pods", "", "default", "p", pod))
    assert pod["spec"].get("tolerations") == want


def test_extended_resource_toleration_sees_resourcev2_gpus():
    """GPU-aware: after ResourceV2 moved `amd.com/gpu` to spec.extendedResources, the pod still
    tolerates the `amd.com/gpu` taint that keeps CPU-only pods off GPU nodes."""
    from kubernetes_amd.api import core
    chain = new_chain(["ResourceV2", "ExtendedResourceToleration"])
    pod = {"metadata": {"name": "g", "namespace": "default"},
           "spec": {"containers": [{"name": "c", "image": "x", "resources": {"limits": {core.AMD_GPU: "2"}}}]}}
    chain.admit(Attributes(CREATE, "pods", "", "default", "g", pod))
    assert pod["spec"]["extendedResources"] and core.AMD_GPU not in pod["spec"]["containers"][0]["resources"].get(
        "limits", {})
    assert pod["spec"]["tolerations"] == [{"key": core.AMD_GPU, "operator": "Exists", "effect": "NoSchedule"}]


def test_extended_resource_toleration_ignores_subresources():
    chain = new_chain(["ExtendedResourceToleration"])
    pod = {"metadata": {"name": "p"}, "spec": {"containers": [ER1_C]}}
    chain.admit(Attributes(CREATE, "pods", "status", "default", "p", pod))
    assert "tolerations" not in pod["spec"]


# -- PodTolerationRestriction: `plugin/pkg/admission/podtolerationrestriction/admission_test.go`

import json as _json  # noqa: E402

from kubernetes_amd.apiserver.admission import UPDATE, AdmissionError  # noqa: E402
from kubernetes_amd.apiserver.admission.security import (MEMORY_PRESSURE_TAINT, PodTolerationRestriction,  # noqa: E402
                                                         merge_tolerations, tolerations_conflict,
                                                         verify_against_whitelist)


class _NsServer:
    def __init__(self, annotations):
        self.ns = {"metadata": {"name": "testNamespace", "annotations": annotations}}

    def get_object(self, resource, namespace, name):
        return self.ns if resource == "namespaces" and name == "testNamespace" else None


def tv(value="testValue", key="testKey"):
    return {"key": key, "operator": "Equal", "value": value, "effect": "NoSchedule"}


MP = {"key": MEMORY_PRESSURE_TAINT, "operator": "Exists", "effect": "NoSchedule"}
BEST_EFFORT = [{"name": "test"}]
BURSTABLE = [{"name": "test", "resources": {"limits": {"cpu": "1000m"}, "requests": {"cpu": "500m"}}}]
GUARANTEED = [{"name": "test", "resources": {"limits": {"cpu": "1000m"}, "requests": {"cpu": "1000m"}}}]

# (name, containers, cluster default, ns default, ns whitelist, cluster whitelist, pod tolerations, merged, admit)
PTR_CASES = [
    ("default cluster tolerations with empty pod tolerations and nil namespace tolerations",
     BEST_EFFORT, [tv()], None, None, None, [], [tv()], True),
    ("default cluster tolerations with pod tolerations specified",
     BEST_EFFORT, [tv()], [], None, None, [tv()], [tv()], True),
    ("namespace tolerations", BEST_EFFORT, [], [tv()], None, None, [tv()], [tv()], True),
    ("no pod tolerations", BEST_EFFORT, [], [tv()], None, None, [], [tv()], True),
    ("conflicting pod and namespace tolerations", BEST_EFFORT, [], [tv()], None, None, [tv("testValue1")], None,
     False),
    ("conflicting pod and default cluster tolerations but overridden by empty namespace tolerations",
     BEST_EFFORT, [tv("testValue2")], [], None, None, [tv("testValue1")], [tv("testValue1")], True),
    ("merged pod tolerations satisfy whitelist", BEST_EFFORT, [], [tv()], [tv()], None, [], [tv()], True),
    ("Override default cluster toleration by empty namespace level toleration",
     BEST_EFFORT, [tv()], [], None, None, [], [], True),
    ("pod toleration conflicts with default cluster white list which is overridden by empty namespace whitelist",
     BEST_EFFORT, None, [], [], [tv("testValue1")], [tv()], [tv()], True),
    ("merged pod tolerations conflict with the whitelist", BEST_EFFORT, [], [tv()], [tv("testValue1")], None, [],
     None, False),
    ("added memoryPressure/DiskPressure for Burstable pod", BURSTABLE, [], [tv()], [], None, [], [MP, tv()], True),
    ("added memoryPressure/DiskPressure for Guaranteed pod", GUARANTEED, [], [tv()], [], None, [], [MP, tv()], True),
]


def _same(a, b):
    """tolerations.EqualTolerations: order-insensitive by (key, effect)."""
    key = lambda t: (t.get("key", ""), t.get("effect", ""))  # noqa: E731
    return len(a) == len(b) and {key(t): t for t in a} == {key(t): t for t in b}


@pytest.mark.parametrize("case", PTR_CASES, ids=[c[0] for c in PTR_CASES])
def test_pod_toleration_restriction(case):
    import copy
    name, ctrs, cdefault, ns_default, ns_wl, cwl, pod_tols, merged, admit = case
    ann = {}
    if ns_default is not None:
        ann[PodTolerationRestriction.DEFAULT] = _json.dumps(ns_default)
    if ns_wl is not None:
        ann[PodTolerationRestriction.WHITELIST] = _json.dumps(ns_wl)
    plugin = PodTolerationRestriction(_NsServer(ann), {"default": cdefault, "whitelist": cwl})
    for op in (CREATE, UPDATE):
        pod = {"metadata": {"name": "testPod", "namespace": "testNamespace"},
               "spec": {"containers": copy.deepcopy(ctrs), "tolerations": copy.deepcopy(pod_tols)}}
        old = None
        if op == UPDATE:   # an update of an uninitialized pod is handled like a create
            old = copy.deepcopy(pod)
            old["metadata"]["initializers"] = {"pending": [{"name": "init"}]}
            old["spec"]["tolerations"] = [tv("testValue1")]
        a = Attributes(op, "pods", "", "testNamespace", "testPod", pod, old)
        if admit:
            plugin.admit(a)
            assert _same(pod["spec"]["tolerations"], merged), (name, op)
        else:
            with pytest.raises(AdmissionError):
                plugin.admit(a)


def test_pod_toleration_restriction_ignores_updating_initialized_pod():
    """TestIgnoreUpdatingInitializedPod: no default merge (and so no conflict) on a plain update."""
    ann = {PodTolerationRestriction.DEFAULT: _json.dumps([tv("testValue2")])}
    plugin = PodTolerationRestriction(_NsServer(ann), {})
    pod = {"metadata": {"name": "testPod", "namespace": "testNamespace"},
           "spec": {"containers": [{"name": "c"}], "tolerations": [tv("testValue1")]}}
    plugin.admit(Attributes(UPDATE, "pods", "", "testNamespace", "testPod", pod, dict(pod)))
    assert pod["spec"]["tolerations"] == [tv("testValue1")]
    assert PodTolerationRestriction(None, {}).handles(CREATE) and PodTolerationRestriction(None, {}).handles(UPDATE)
    assert not PodTolerationRestriction(None, {}).handles("DELETE")


def test_toleration_set_helpers():
    assert tolerations_conflict([tv("a")], [tv("b")]) and not tolerations_conflict([tv("a")], [tv("a")])
    assert not tolerations_conflict([tv("a", key="k1")], [tv("b", key="k2")])
    assert merge_tolerations([tv("a"), tv("x", key="k2")], [tv("b")]) == [tv("b"), tv("x", key="k2")]
    assert verify_against_whitelist([tv()], []) and verify_against_whitelist([tv()], [tv(), tv(key="o")])
    assert not verify_against_whitelist([tv("other")], [tv()])
