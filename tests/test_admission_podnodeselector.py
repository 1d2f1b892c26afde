"""PodNodeSelector admission — port of `plugin/pkg/admission/podnodeselector/admission_test.go`
(TestPodAdmission: cluster default selector, namespace annotation with whitespace, empty
annotation, conflicts, whitelist; create and update of an uninitialized pod; IgnoreUpdate of
an initialized pod; subresources ignored)."""
import pytest

from kubernetes_amd.apiserver.admission import CREATE, UPDATE, AdmissionError, Attributes, new_chain

ANN = "scheduler.alpha.kubernetes.io/node-selector"


class FakeServer:
    def __init__(self):
        self.ns = {"metadata": {"name": "testNamespace"}}

    def get_object(self, resource, namespace, name):
        return self.ns if resource == "namespaces" and name == "testNamespace" else None


CASES = [
    # default, namespace annotation (None: leave as is), whitelist, pod selector, merged, admit
    ("", None, "", {}, {}, True, "No node selectors"),
    ("infra = false", None, "", {}, {"infra": "false"}, True, "Default node selector and no conflicts"),
    ("", " infra = false ", "", {}, {"infra": "false"}, True, "Namespace node selector with whitespaces"),
    ("infra = false", "infra=true", "", {}, {"infra": "true"}, True, "Default and namespace node selector"),
    ("infra = false", "", "", {}, {}, True, "Empty namespace node selector and no conflicts"),
    ("infra = false", "infra=true", "", {"env": "test"}, {"infra": "true", "env": "test"}, True,
     "Namespace and pod node selector, no conflicts"),
    ("env = test", "infra=true", "", {"infra": "false"}, None, False, "Conflicting pod and namespace selector, one label"),
    ("env=dev", "infra=false, env = test", "", {"env": "dev", "color": "blue"}, None, False,
     "Conflicting pod and namespace node selector, multiple labels"),
    ("env=dev", "infra=false, env = dev", "env=dev, infra=false, color=blue", {"env": "dev", "color": "blue"},
     {"infra": "false", "env": "dev", "color": "blue"}, True, "Merged pod node selectors satisfy the whitelist"),
    ("env=dev", "infra=false, env = dev", "env=dev, infra=true, color=blue", {"env": "dev", "color": "blue"}, None,
     False, "Merged pod node selectors conflict with the whitelist"),
    ("env=dev", None, "env=prd", {}, None, False, "Default node selector conflict with the whitelist"),
]


def test_pod_admission_table():
    srv = FakeServer()
    for default, ns_sel, white, pod_sel, merged, ok, name in CASES:
        if ns_sel is not None:
            srv.ns["metadata"]["annotations"] = {ANN: ns_sel}
        chain = new_chain(["PodNodeSelector"], srv, {"PodNodeSelector": {"podNodeSelectorPluginConfig": {
            "clusterDefaultNodeSelector": default, "testNamespace": white}}})
        old = {"metadata": {"name": "testPod", "namespace": "testNamespace",
                            "initializers": {"pending": [{"name": "init"}]}}, "spec": {"nodeSelector": {"old": "true"}}}
        for op, prev in ((CREATE, None), (UPDATE, old)):      # an uninitialized pod's update is a create
            pod = {"metadata": {"name": "testPod", "namespace": "testNamespace"}, "spec": {"nodeSelector": dict(pod_sel)}}
            a = Attributes(op, "pods", "", "testNamespace", "testPod", pod, prev)
            try:
                chain.admit(a)
                chain.validate(a)
                got = True
            except AdmissionError:
                got = False
            assert got == ok, (name, op)
            if ok:
                assert (pod["spec"].get("nodeSelector") or {}) == merged, (name, op)


def test_ignores_updates_of_initialized_pods_and_subresources():
    srv = FakeServer()
    srv.ns["metadata"]["annotations"] = {ANN: "infra=true"}
    chain = new_chain(["PodNodeSelector"], srv)
    old = {"metadata": {"name": "p", "namespace": "testNamespace"}, "spec": {"nodeSelector": {"old": "true"}}}
    pod = {"metadata": {"name": "p", "namespace": "testNamespace"}, "spec": {"nodeSelector": {"old": "true"}}}
    chain.admit(Attributes(UPDATE, "pods", "", "testNamespace", "p", pod, old))
    assert pod["spec"]["nodeSelector"] == {"old": "true"}
    chain.admit(Attributes(CREATE, "pods", "binding", "testNamespace", "p", {"target": {}}, None))
    with pytest.raises(AdmissionError, match="invalid selector"):     # an unparsable whitelist
        new_chain(["PodNodeSelector"], srv, {"PodNodeSelector": {"podNodeSelectorPluginConfig": {
            "testNamespace": "novalue"}}}).validate(Attributes(CREATE, "pods", "", "testNamespace", "p", pod, None))
