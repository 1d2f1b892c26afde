"""Priority admission — port of `plugin/pkg/admission/priority/admission_test.go`
(TestPriorityClassAdmission, TestPodAdmission; TestDefaultPriority's resolution cases)."""
import pytest

from kubernetes_amd.apiserver.admission import CREATE, UPDATE, AdmissionError, Attributes, new_chain
from kubernetes_amd.apiserver.admission.plugins import SYSTEM_CRITICAL_PRIORITY


def pc(name, value, default=False):
    return {"kind": "PriorityClass", "metadata": {"name": name}, "value": value, "globalDefault": default}


DEFAULT1, DEFAULT2, NONDEFAULT1 = pc("default1", 1000, True), pc("default2", 2000, True), pc("nondefault1", 2000)


class FakeServer:
    def __init__(self, classes):
        self.classes = list(classes)

    def list_objects(self, resource, namespace=None):
        return self.classes if resource == "priorityclasses" else []

    def get_object(self, resource, namespace, name):
        return next((c for c in self.list_objects(resource) if c["metadata"]["name"] == name), None)


def run(classes, op, resource, obj, old=None):
    chain = new_chain(["Priority"], FakeServer(classes))
    a = Attributes(op, resource, "", "namespace", obj["metadata"]["name"], obj, old)
    chain.admit(a)
    chain.validate(a)
    return obj


@pytest.mark.parametrize("name,existing,cls,err", [
    ("one default class", [], DEFAULT1, False),
    ("more than one default classes", [DEFAULT1], DEFAULT2, True),
    ("too high PriorityClass value", [], pc("toohighclass", 1000000001), True),
    ("system name conflict", [], pc("system-cluster-critical", 2000000000), True),
])
def test_priority_class_admission(name, existing, cls, err):
    if err:
        with pytest.raises(AdmissionError):
            run(existing, CREATE, "priorityclasses", dict(cls))
    else:
        run(existing, CREATE, "priorityclasses", dict(cls))


def test_marking_the_default_class_again_or_another():
    run([DEFAULT1], UPDATE, "priorityclasses", dict(DEFAULT1, value=3), DEFAULT1)     # the default itself
    with pytest.raises(AdmissionError, match="default1 is already marked as default"):
        run([DEFAULT1, NONDEFAULT1], UPDATE, "priorityclasses", dict(NONDEFAULT1, globalDefault=True), NONDEFAULT1)


def pod(name, pcn=None, priority=None, mirror=False):
    md = {"name": name, "namespace": "namespace"}
    if mirror:
        md["annotations"] = {"kubernetes.io/config.mirror": ""}
    spec = {"containers": [{"name": "c"}]}
    if pcn:
        spec["priorityClassName"] = pcn
    if priority is not None:
        spec["priority"] = priority
    return {"metadata": md, "spec": spec}


@pytest.mark.parametrize("name,existing,p,want", [
    ("Pod with priority class", [DEFAULT1, NONDEFAULT1], pod("pod-w-priorityclass", "default1"), 1000),
    ("Pod without priority class", [DEFAULT1], pod("pod-wo-priorityclass"), 1000),
    ("pod without priority class and no existing priority class", [], pod("pod-wo-priorityclass"), 0),
    ("pod without priority class and no default class", [NONDEFAULT1], pod("pod-wo-priorityclass"), 0),
    ("pod with a system priority class", [], pod("pod-w-system-priority", "system-cluster-critical"),
     SYSTEM_CRITICAL_PRIORITY),
    ("Pod with non-existing priority class", [DEFAULT1, NONDEFAULT1], pod("p", "non-existing"), None),
    ("pod with integer priority", [], pod("pod-w-integer-priority", "default1", 1000), None),
    ("mirror pod with system priority class", [], pod("m", "system-cluster-critical", mirror=True),
     SYSTEM_CRITICAL_PRIORITY),
    ("mirror pod with integer priority", [], pod("m", "default1", 1000, mirror=True), None),
])
def test_pod_admission(name, existing, p, want):
    if want is None:
        with pytest.raises(AdmissionError):
            run(existing, CREATE, "pods", p)
    else:
        assert run(existing, CREATE, "pods", p)["spec"]["priority"] == want


def test_default_priority_follows_the_classes():
    assert run([DEFAULT1], CREATE, "pods", pod("a"))["spec"]["priority"] == 1000
    assert run([NONDEFAULT1], CREATE, "pods", pod("a"))["spec"]["priority"] == 0       # default deleted
    assert run([dict(DEFAULT1, globalDefault=False)], CREATE, "pods", pod("a"))["spec"]["priority"] == 0
    # updates of pods are not re-resolved (pod validation keeps priority immutable)
    p = pod("a", priority=5)
    run([DEFAULT1], UPDATE, "pods", p, pod("a", priority=5))
    assert p["spec"]["priority"] == 5
