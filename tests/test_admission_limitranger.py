"""LimitRanger and ServiceAccount admission.

Ported tables: `plugin/pkg/admission/limitranger/admission_test.go` (TestDefaultContainer-
ResourceRequirements :162, TestMergePodResourceRequirements :193, TestPodLimitFunc :255 — all
success and error cases, TestPodLimitFuncApplyDefault :636, TestLimitRangerIgnoresSubresource
:687, TestLimitRangerAdmitPod :713, TestPersistentVolumeClaimLimitFunc :779) and
`plugin/pkg/admission/serviceaccount/admission_test.go` (mirror pods :83-139, default account
:141, denied / required account and token :169-239, AllowsReferencedSecret :504,
RejectsUnreferencedSecretVolumes :585, AllowUnreferencedSecretVolumesForPermissiveSAs :663,
Allows/RejectsReferencedImagePullSecrets :695-755, Do/AddImagePullSecrets :756-831). GPU cases
(ResourceV2-moved `amd.com/gpu` seen by the constraints) are MI355X additions.
"""
import pytest

from kubernetes_amd.api import core
from kubernetes_amd.apiserver.admission import CREATE, UPDATE, AdmissionError, Attributes, new_chain
from kubernetes_amd.apiserver.admission.limitranger import (LIMIT_RANGER_ANNOTATION, default_container_requirements,
                                                           merge_pod_resource_requirements, pod_mutate_limit,
                                                           pod_validate_limit, pvc_validate_limit)
from kubernetes_amd.apiserver.server import APIServer
from kubernetes_amd.client.rest import APIStatusError, Client


def rl(cpu="", mem=""):
    out = {}
    if cpu:
        out["cpu"] = cpu
    if mem:
        out["memory"] = mem
    return out


def eph(v=""):
    return {"ephemeral-storage": v} if v else {}


def storage(v=""):
    return {"storage": v} if v else {}


def rr(requests, limits):
    return {"requests": dict(requests), "limits": dict(limits)}


def limit_range(kind, mn=None, mx=None, default=None, default_request=None, ratio=None):
    item = {"type": kind}
    for k, v in (("min", mn), ("max", mx), ("default", default), ("defaultRequest", default_request),
                 ("maxLimitRequestRatio", ratio)):
        if v:
            item[k] = v
    return {"metadata": {"name": "abc", "namespace": "test"}, "spec": {"limits": [item]}}


def valid_limit_range(defaults=True):
    ctr = {"type": "Container", "max": rl("100m", "2Gi"), "min": rl("25m", "1Mi")}
    if defaults:
        ctr.update({"default": rl("75m", "10Mi"), "defaultRequest": rl("50m", "5Mi")})
    return {"metadata": {"name": "abc", "namespace": "test"},
            "spec": {"limits": [{"type": "Pod", "max": rl("200m", "4Gi"), "min": rl("50m", "2Mi")}, ctr]}}


def valid_pod(name, n, res):
    return {"metadata": {"name": name, "namespace": "test"},
            "spec": {"containers": [{"name": f"foo-{i}", "image": f"foo:V{i}",
                                     "resources": {k: dict(v) for k, v in res.items()}} for i in range(n)]}}


def with_init(pod, *resources):
    pod["spec"]["initContainers"] = [{"name": f"foo-{i}", "image": f"foo:V{i}",
                                      "resources": {k: dict(v) for k, v in r.items()}} for i, r in enumerate(resources)]
    return pod


C, P = "Container", "Pod"

SUCCESS = [
    (valid_pod("ctr-min-cpu-request", 1, rr(rl("100m"), {})), limit_range(C, mn=rl("50m"))),
    (valid_pod("ctr-min-cpu-request-limit", 1, rr(rl("100m"), rl("200m"))), limit_range(C, mn=rl("50m"))),
    (valid_pod("ctr-min-memory-request", 1, rr(rl(mem="60Mi"), {})), limit_range(C, mn=rl(mem="50Mi"))),
    (valid_pod("ctr-min-memory-request-limit", 1, rr(rl(mem="60Mi"), rl(mem="100Mi"))), limit_range(C, mn=rl(mem="50Mi"))),
    (valid_pod("ctr-max-cpu-request-limit", 1, rr(rl("500m"), rl("1"))), limit_range(C, mx=rl("2"))),
    (valid_pod("ctr-max-cpu-limit", 1, rr({}, rl("1"))), limit_range(C, mx=rl("2"))),
    (valid_pod("ctr-max-mem-request-limit", 1, rr(rl(mem="250Mi"), rl(mem="500Mi"))), limit_range(C, mx=rl(mem="1Gi"))),
    (valid_pod("ctr-max-cpu-ratio", 1, rr(rl("500m"), rl("750m"))), limit_range(C, ratio=rl("1.5"))),
    (valid_pod("ctr-max-mem-limit", 1, rr({}, rl(mem="500Mi"))), limit_range(C, mx=rl(mem="1Gi"))),
    (valid_pod("pod-min-cpu-request", 2, rr(rl("75m"), {})), limit_range(P, mn=rl("100m"))),
    (valid_pod("pod-min-cpu-request-limit", 2, rr(rl("75m"), rl("200m"))), limit_range(P, mn=rl("100m"))),
    (valid_pod("pod-min-memory-request", 2, rr(rl(mem="60Mi"), {})), limit_range(P, mn=rl(mem="100Mi"))),
    (valid_pod("pod-min-memory-request-limit", 2, rr(rl(mem="60Mi"), rl(mem="100Mi"))), limit_range(P, mn=rl(mem="100Mi"))),
    (with_init(valid_pod("pod-init-min-memory-request", 2, rr(rl(mem="60Mi"), {})), rr(rl(mem="100Mi"), {})),
     limit_range(P, mn=rl(mem="100Mi"))),
    (with_init(valid_pod("pod-init-min-memory-request-limit", 2, rr(rl(mem="60Mi"), rl(mem="100Mi"))),
               rr(rl(mem="80Mi"), rl(mem="100Mi"))), limit_range(P, mn=rl(mem="100Mi"))),
    (valid_pod("pod-max-cpu-request-limit", 2, rr(rl("500m"), rl("1"))), limit_range(P, mx=rl("2"))),
    (valid_pod("pod-max-cpu-limit", 2, rr({}, rl("1"))), limit_range(P, mx=rl("2"))),
    (with_init(valid_pod("pod-init-max-cpu-request-limit", 2, rr(rl("500m"), rl("1"))), rr(rl("1"), rl("2")),
               rr(rl("1"), rl("1"))), limit_range(P, mx=rl("2"))),
    (with_init(valid_pod("pod-init-max-cpu-limit", 2, rr({}, rl("1"))), rr({}, rl("2")), rr({}, rl("2"))),
     limit_range(P, mx=rl("2"))),
    (valid_pod("pod-max-mem-request-limit", 2, rr(rl(mem="250Mi"), rl(mem="500Mi"))), limit_range(P, mx=rl(mem="1Gi"))),
    (valid_pod("pod-max-mem-limit", 2, rr({}, rl(mem="500Mi"))), limit_range(P, mx=rl(mem="1Gi"))),
    (valid_pod("pod-max-mem-ratio", 3, rr(rl(mem="300Mi"), rl(mem="450Mi"))),
     limit_range(P, mx=rl(mem="2Gi"), ratio=rl(mem="1.5"))),
    (valid_pod("ctr-1-min-eph-request", 1, rr(eph("60Mi"), {})), limit_range(C, mn=eph("50Mi"))),
    (valid_pod("ctr-1-min-eph-request-limit", 1, rr(eph("60Mi"), eph("100Mi"))), limit_range(C, mn=eph("50Mi"))),
    (valid_pod("ctr-1-max-eph-request-limit", 1, rr(eph("250Mi"), eph("500Mi"))), limit_range(C, mx=eph("1Gi"))),
    (valid_pod("ctr-1-max-eph-limit", 1, rr({}, eph("500Mi"))), limit_range(C, mx=eph("1Gi"))),
    (valid_pod("ctr-2-min-eph-request", 2, rr(eph("60Mi"), {})), limit_range(C, mn=eph("50Mi"))),
    (valid_pod("ctr-2-min-eph-request-limit", 2, rr(eph("60Mi"), eph("100Mi"))), limit_range(C, mn=eph("50Mi"))),
    (valid_pod("ctr-2-max-eph-request-limit", 2, rr(eph("250Mi"), eph("500Mi"))), limit_range(C, mx=eph("600Mi"))),
    (valid_pod("ctr-2-max-eph-limit", 2, rr({}, eph("500Mi"))), limit_range(C, mx=eph("600Mi"))),
    (valid_pod("pod-min-eph-request", 2, rr(eph("60Mi"), {})), limit_range(P, mn=eph("100Mi"))),
    (valid_pod("pod-min-eph-request-limit", 2, rr(eph("60Mi"), eph("100Mi"))), limit_range(P, mn=eph("100Mi"))),
    (with_init(valid_pod("pod-init-min-eph-request", 2, rr(eph("60Mi"), {})), rr(eph("100Mi"), {})),
     limit_range(P, mn=eph("100Mi"))),
    (with_init(valid_pod("pod-init-min-eph-request-limit", 2, rr(eph("60Mi"), eph("100Mi"))),
               rr(eph("80Mi"), eph("100Mi"))), limit_range(P, mn=eph("100Mi"))),
    (valid_pod("pod-max-eph-request-limit", 2, rr(eph("250Mi"), eph("500Mi"))), limit_range(P, mx=eph("1Gi"))),
    (valid_pod("pod-max-eph-limit", 2, rr({}, eph("500Mi"))), limit_range(P, mx=eph("1Gi"))),
    (valid_pod("pod-max-eph-ratio", 3, rr(eph("300Mi"), eph("450Mi"))), limit_range(P, mx=eph("2Gi"), ratio=eph("1.5"))),
]

ERRORS = [
    (valid_pod("ctr-min-cpu-request", 1, rr(rl("40m"), {})), limit_range(C, mn=rl("50m"))),
    (valid_pod("ctr-min-cpu-request-limit", 1, rr(rl("40m"), rl("200m"))), limit_range(C, mn=rl("50m"))),
    (valid_pod("ctr-min-cpu-no-request-limit", 1, rr({}, {})), limit_range(C, mn=rl("50m"))),
    (valid_pod("ctr-min-memory-request", 1, rr(rl(mem="40Mi"), {})), limit_range(C, mn=rl(mem="50Mi"))),
    (valid_pod("ctr-min-memory-request-limit", 1, rr(rl(mem="40Mi"), rl(mem="100Mi"))), limit_range(C, mn=rl(mem="50Mi"))),
    (valid_pod("ctr-min-memory-no-request-limit", 1, rr({}, {})), limit_range(C, mn=rl(mem="50Mi"))),
    (valid_pod("ctr-max-cpu-request-limit", 1, rr(rl("500m"), rl("2500m"))), limit_range(C, mx=rl("2"))),
    (valid_pod("ctr-max-cpu-limit", 1, rr({}, rl("2500m"))), limit_range(C, mx=rl("2"))),
    (valid_pod("ctr-max-cpu-no-request-limit", 1, rr({}, {})), limit_range(C, mx=rl("2"))),
    (valid_pod("ctr-max-cpu-ratio", 1, rr(rl("1250m"), rl("2500m"))), limit_range(C, ratio=rl("1"))),
    (valid_pod("ctr-max-mem-request-limit", 1, rr(rl(mem="250Mi"), rl(mem="2Gi"))), limit_range(C, mx=rl(mem="1Gi"))),
    (valid_pod("ctr-max-mem-limit", 1, rr({}, rl(mem="2Gi"))), limit_range(C, mx=rl(mem="1Gi"))),
    (valid_pod("ctr-max-mem-no-request-limit", 1, rr({}, {})), limit_range(C, mx=rl(mem="1Gi"))),
    (valid_pod("pod-min-cpu-request", 1, rr(rl("75m"), {})), limit_range(P, mn=rl("100m"))),
    (valid_pod("pod-min-cpu-request-limit", 1, rr(rl("75m"), rl("200m"))), limit_range(P, mn=rl("100m"))),
    (valid_pod("pod-min-memory-request", 1, rr(rl(mem="60Mi"), {})), limit_range(P, mn=rl(mem="100Mi"))),
    (valid_pod("pod-min-memory-request-limit", 1, rr(rl(mem="60Mi"), rl(mem="100Mi"))), limit_range(P, mn=rl(mem="100Mi"))),
    (valid_pod("pod-max-cpu-request-limit", 3, rr(rl("500m"), rl("1"))), limit_range(P, mx=rl("2"))),
    (valid_pod("pod-max-cpu-limit", 3, rr({}, rl("1"))), limit_range(P, mx=rl("2"))),
    (valid_pod("pod-max-mem-request-limit", 3, rr(rl(mem="250Mi"), rl(mem="500Mi"))), limit_range(P, mx=rl(mem="1Gi"))),
    (valid_pod("pod-max-mem-limit", 3, rr({}, rl(mem="500Mi"))), limit_range(P, mx=rl(mem="1Gi"))),
    (with_init(valid_pod("pod-init-max-mem-limit", 1, rr({}, rl(mem="500Mi"))), rr({}, rl(mem="1.5Gi"))),
     limit_range(P, mx=rl(mem="1Gi"))),
    (valid_pod("pod-max-mem-ratio", 3, rr(rl(mem="250Mi"), rl(mem="500Mi"))),
     limit_range(P, mx=rl(mem="2Gi"), ratio=rl(mem="1.5"))),
    (valid_pod("ctr-1-min-eph-request", 1, rr(eph("40Mi"), {})), limit_range(C, mn=eph("50Mi"))),
    (valid_pod("ctr-1-min-eph-request-limit", 1, rr(eph("40Mi"), eph("100Mi"))), limit_range(C, mn=eph("50Mi"))),
    (valid_pod("ctr-1-min-eph-no-request-limit", 1, rr({}, {})), limit_range(C, mn=eph("50Mi"))),
    (valid_pod("ctr-1-max-eph-request-limit", 1, rr(eph("250Mi"), eph("2Gi"))), limit_range(C, mx=eph("1Gi"))),
    (valid_pod("ctr-1-max-eph-limit", 1, rr({}, eph("2Gi"))), limit_range(C, mx=eph("1Gi"))),
    (valid_pod("ctr-1-max-eph-no-request-limit", 1, rr({}, {})), limit_range(C, mx=eph("1Gi"))),
    (valid_pod("ctr-2-min-eph-request", 2, rr(eph("40Mi"), {})), limit_range(C, mn=eph("50Mi"))),
    (valid_pod("ctr-2-min-eph-request-limit", 2, rr(eph("40Mi"), eph("100Mi"))), limit_range(C, mn=eph("50Mi"))),
    (valid_pod("ctr-2-min-eph-no-request-limit", 2, rr({}, {})), limit_range(C, mn=eph("50Mi"))),
    (valid_pod("ctr-2-max-eph-request-limit", 2, rr(eph("250Mi"), eph("2Gi"))), limit_range(C, mx=eph("1Gi"))),
    (valid_pod("ctr-2-max-eph-limit", 2, rr({}, eph("2Gi"))), limit_range(C, mx=eph("1Gi"))),
    (valid_pod("ctr-2-max-eph-no-request-limit", 2, rr({}, {})), limit_range(C, mx=eph("1Gi"))),
    (valid_pod("pod-min-eph-request", 1, rr(eph("60Mi"), {})), limit_range(P, mn=eph("100Mi"))),
    (valid_pod("pod-min-eph-request-limit", 1, rr(eph("60Mi"), eph("100Mi"))), limit_range(P, mn=eph("100Mi"))),
    (valid_pod("pod-max-eph-request-limit", 3, rr(eph("250Mi"), eph("500Mi"))), limit_range(P, mx=eph("1Gi"))),
    (valid_pod("pod-max-eph-limit", 3, rr({}, eph("500Mi"))), limit_range(P, mx=eph("1Gi"))),
    (with_init(valid_pod("pod-init-max-eph-limit", 1, rr({}, eph("500Mi"))), rr({}, eph("1.5Gi"))),
     limit_range(P, mx=eph("1Gi"))),
    (valid_pod("pod-max-eph-ratio", 3, rr(eph("250Mi"), eph("500Mi"))), limit_range(P, mx=eph("2Gi"), ratio=eph("1.5"))),
]


@pytest.mark.parametrize("pod,lr", SUCCESS, ids=[p["metadata"]["name"] for p, _ in SUCCESS])
def test_pod_limit_func_success(pod, lr):
    pod_mutate_limit(lr, pod)
    assert pod_validate_limit(lr, pod) == []


@pytest.mark.parametrize("pod,lr", ERRORS, ids=[p["metadata"]["name"] for p, _ in ERRORS])
def test_pod_limit_func_errors(pod, lr):
    pod_mutate_limit(lr, pod)
    assert pod_validate_limit(lr, pod)


def test_error_strings_match_reference():
    lr = limit_range(C, mn=rl("50m"))
    assert pod_validate_limit(lr, valid_pod("a", 1, rr({}, {}))) == [
        "minimum cpu usage per Container is 50m.  No request is specified."]
    assert pod_validate_limit(lr, valid_pod("a", 1, rr(rl("40m"), {}))) == [
        "minimum cpu usage per Container is 50m, but request is 40m."]
    lr = limit_range(C, mx=rl(mem="1Gi"))
    assert pod_validate_limit(lr, valid_pod("a", 1, rr({}, {}))) == [
        "maximum memory usage per Container is 1Gi.  No limit is specified."]
    assert pod_validate_limit(lr, valid_pod("a", 1, rr({}, rl(mem="2Gi")))) == [
        "maximum memory usage per Container is 1Gi, but limit is 2Gi."]
    lr = limit_range(C, ratio=rl("1"))
    assert pod_validate_limit(lr, valid_pod("a", 1, rr(rl("1250m"), rl("2500m")))) == [
        "cpu max limit to request ratio per Container is 1, but provided ratio is 2.000000."]
    assert pod_validate_limit(lr, valid_pod("a", 1, rr({}, rl("1")))) == [
        "cpu max limit to request ratio per Container is 1, but no request is specified or request is 0."]


def test_default_container_resource_requirements():
    assert default_container_requirements(valid_limit_range()) == (rl("50m", "5Mi"), rl("75m", "10Mi"))


def test_merge_pod_resource_requirements():
    defaults = default_container_requirements(valid_limit_range())
    pod = valid_pod("empty-resources", 1, rr({}, {}))
    merge_pod_resource_requirements(pod, defaults)
    assert pod["spec"]["containers"][0]["resources"] == {"requests": rl("50m", "5Mi"), "limits": rl("75m", "10Mi")}
    assert pod["metadata"]["annotations"][LIMIT_RANGER_ANNOTATION] == (
        "LimitRanger plugin set: cpu, memory request for container foo-0; cpu, memory limit for container foo-0")
    inp = rr(rl(mem="512Mi"), {})
    pod = with_init(valid_pod("limit-memory", 1, inp), inp)
    merge_pod_resource_requirements(pod, defaults)
    want = {"requests": {"cpu": "50m", "memory": "512Mi"}, "limits": rl("75m", "10Mi")}
    assert pod["spec"]["containers"][0]["resources"] == want
    assert pod["spec"]["initContainers"][0]["resources"] == want
    # the reference's table expects only the container entries: its container and init
    # container share one Go map (`input`), so the init container looks already defaulted. With
    # independent resources the init container is defaulted and annotated as well.
    assert pod["metadata"]["annotations"][LIMIT_RANGER_ANNOTATION] == (
        "LimitRanger plugin set: cpu request for container foo-0; cpu, memory limit for container foo-0; "
        "cpu request for init container foo-0; cpu, memory limit for init container foo-0")
    inp = rr(rl("100m", "512Mi"), rl("200m", "1G"))
    init = rr(rl("200m", "1G"), rl("400m", "2G"))
    pod = with_init(valid_pod("limit-memory", 1, inp), init)
    merge_pod_resource_requirements(pod, defaults)
    assert pod["spec"]["containers"][0]["resources"] == inp
    assert pod["spec"]["initContainers"][0]["resources"] == init
    assert LIMIT_RANGER_ANNOTATION not in (pod["metadata"].get("annotations") or {})


def test_pod_limit_func_apply_default():
    pod = with_init(valid_pod("foo", 1, rr({}, {})), rr({}, {}))
    pod_mutate_limit(valid_limit_range(), pod)
    for c in pod["spec"]["containers"] + pod["spec"]["initContainers"]:
        assert c["resources"] == {"requests": {"cpu": "50m", "memory": "5Mi"}, "limits": {"cpu": "75m", "memory": "10Mi"}}


PVC_OK = [("pvc-is-min", "1Gi", limit_range("PersistentVolumeClaim", mn=storage("1Gi"))),
          ("pvc-is-max", "1Gi", limit_range("PersistentVolumeClaim", mx=storage("1Gi"))),
          ("pvc-no-minmax", "100Gi", limit_range("PersistentVolumeClaim")),
          ("pvc-within-minmax", "5Gi", limit_range("PersistentVolumeClaim", mn=storage("1Gi"), mx=storage("10Gi")))]
PVC_BAD = [("pvc-below-min", "500Mi", limit_range("PersistentVolumeClaim", mn=storage("1Gi"))),
           ("pvc-exceeds-max", "100Gi", limit_range("PersistentVolumeClaim", mn=storage("1Gi"), mx=storage("1Gi")))]


def _pvc(name, size):
    return {"metadata": {"name": name, "namespace": "test"}, "spec": {"resources": {"requests": storage(size)}}}


def test_persistent_volume_claim_limit_func():
    for name, size, lr in PVC_OK:
        assert pvc_validate_limit(lr, _pvc(name, size)) == [], name
    for name, size, lr in PVC_BAD:
        assert pvc_validate_limit(lr, _pvc(name, size)), name


class FakeServer:
    def __init__(self, **objs):
        self.objs = objs

    def list_objects(self, resource, namespace=None):
        return [o for o in self.objs.get(resource, ()) if namespace is None or o["metadata"].get("namespace") == namespace]

    def get_object(self, resource, namespace, name):
        for o in self.list_objects(resource, namespace):
            if o["metadata"]["name"] == name:
                return o
        return None


def _attrs(op, obj, resource="pods", sub="", ns="test"):
    return Attributes(op, resource, sub, ns, obj["metadata"]["name"], obj)


def test_limit_ranger_admit_pod_update_and_subresource():
    chain = new_chain(["LimitRanger"], FakeServer(limitranges=[valid_limit_range(defaults=False)]))
    pod = valid_pod("testPod", 1, {})
    chain.admit(_attrs(UPDATE, pod))                  # no defaults on update
    assert "requests" not in pod["spec"]["containers"][0]["resources"]
    with pytest.raises(AdmissionError) as e:
        chain.validate(_attrs(UPDATE, pod))
    assert str(e.value).startswith('pods "testPod" is forbidden: [')
    chain.validate(_attrs(UPDATE, pod, sub="status"))  # subresources are ignored


def test_limit_ranger_create_defaults_then_validates():
    chain = new_chain(["LimitRanger"], FakeServer(limitranges=[valid_limit_range()]))
    pod = valid_pod("p", 1, {})
    a = _attrs(CREATE, pod)
    chain.admit(a)
    chain.validate(a)
    assert pod["spec"]["containers"][0]["resources"]["limits"] == rl("75m", "10Mi")
    assert LIMIT_RANGER_ANNOTATION in pod["metadata"]["annotations"]
    big = valid_pod("big", 1, rr(rl("150m"), rl("150m")))
    a = _attrs(CREATE, big)
    chain.admit(a)
    with pytest.raises(AdmissionError, match="maximum cpu usage per Container is 100m, but limit is 150m"):
        chain.validate(a)


def gpu_pod(name, n):
    return {"metadata": {"name": name, "namespace": "test"},
            "spec": {"containers": [{"name": "c", "image": "x", "resources": {"limits": {core.AMD_GPU: str(n)}}}]}}


def test_gpu_limits_are_seen_after_resourcev2():
    """LimitRange{max: {amd.com/gpu: 2}} refuses a 4-GPU pod although ResourceV2 moved the GPU
    limit out of the container into spec.extendedResources."""
    for kind in (C, P):
        lr = limit_range(kind, mx={core.AMD_GPU: "2"})
        chain = new_chain(["LimitRanger", "ResourceV2"], FakeServer(limitranges=[lr]))
        ok = gpu_pod("two", 2)
        a = _attrs(CREATE, ok)
        chain.admit(a)
        assert core.AMD_GPU not in ok["spec"]["containers"][0]["resources"]["limits"]
        chain.validate(a)
        bad = gpu_pod("four", 4)
        a = _attrs(CREATE, bad)
        chain.admit(a)
        with pytest.raises(AdmissionError, match=f"maximum {core.AMD_GPU} usage per {kind} is 2, but limit is 4"):
            chain.validate(a)
    # a defaulted GPU limit is converted by ResourceV2 like a written one
    lr = limit_range(C, default={core.AMD_GPU: "1"})
    chain = new_chain(["LimitRanger", "ResourceV2"], FakeServer(limitranges=[lr]))
    pod = valid_pod("dflt", 1, {})
    a = _attrs(CREATE, pod)
    chain.admit(a)
    assert [core.pod_extended_resource_count(per) for per in pod["spec"]["extendedResources"]] == [1]


def test_limit_ranger_end_to_end(run):
    async def main():
        s = APIServer(admission_plugins=["NamespaceLifecycle", "LimitRanger", "ResourceV2"])
        port = await s.start()
        c = Client(f"http://127.0.0.1:{port}")
        try:
            await c.create("limitranges", {"metadata": {"name": "gpu", "namespace": "default"}, "spec": {"limits": [
                {"type": "Container", "max": {core.AMD_GPU: "2"}, "default": {"cpu": "1"}, "defaultRequest": {"cpu": "500m"}},
                {"type": "PersistentVolumeClaim", "max": {"storage": "1Gi"}}]}})
            p = await c.create("pods", {"metadata": {"name": "ok"}, "spec": {"containers": [
                {"name": "c", "image": "x", "resources": {"limits": {core.AMD_GPU: "2"}}}]}})
            assert p["spec"]["containers"][0]["resources"]["requests"]["cpu"] == "500m"
            assert "cpu request for container c" in p["metadata"]["annotations"][LIMIT_RANGER_ANNOTATION]
            with pytest.raises(APIStatusError) as e:
                await c.create("pods", {"metadata": {"name": "greedy"}, "spec": {"containers": [
                    {"name": "c", "image": "x", "resources": {"limits": {core.AMD_GPU: "4"}}}]}})
            assert e.value.code == 403 and "maximum amd.com/gpu usage per Container is 2" in str(e.value)
            with pytest.raises(APIStatusError) as e:
                await c.create("persistentvolumeclaims", {"metadata": {"name": "big"}, "spec": {
                    "accessModes": ["ReadWriteOnce"], "resources": {"requests": {"storage": "5Gi"}}}})
            assert "maximum storage usage per PersistentVolumeClaim is 1Gi, but request is 5Gi" in str(e.value)
            # an update of the existing pod does not re-default it
            p["metadata"].setdefault("labels", {})["x"] = "y"
            await c.update("pods", p)
        finally:
            await s.stop()
    run(main())


# -- ServiceAccount --------------------------------------------------------------------------------

def sa(name="default", ns="myns", secrets=(), pull=(), enforce=None, automount=None):
    o = {"metadata": {"name": name, "namespace": ns}, "secrets": [{"name": s} for s in secrets],
         "imagePullSecrets": [{"name": s} for s in pull]}
    if enforce is not None:
        o["metadata"]["annotations"] = {"kubernetes.io/enforce-mountable-secrets": enforce}
    if automount is not None:
        o["automountServiceAccountToken"] = automount
    return o


def token(name, ns="myns", sa_name="default"):
    return {"metadata": {"name": name, "namespace": ns, "annotations": {"kubernetes.io/service-account.name": sa_name}},
            "type": "kubernetes.io/service-account-token"}


def sapod(name="myname", ns="myns", **spec):
    return {"metadata": {"name": name, "namespace": ns}, "spec": dict({"containers": [{"name": "c"}]}, **spec)}


def run_chain(server, pod, config=None, ns="myns"):
    chain = new_chain(["ServiceAccount"], server, {"ServiceAccount": config} if config else None)
    a = Attributes(CREATE, "pods", "", ns, pod["metadata"]["name"], pod)
    chain.admit(a)
    chain.validate(a)
    return pod


MIRROR = {"kubernetes.io/config.mirror": "true"}


def test_mirror_pods():
    ok = {"metadata": {"name": "m", "annotations": dict(MIRROR)}, "spec": {"volumes": [{"name": "v", "emptyDir": {}}]}}
    run_chain(FakeServer(), ok)
    assert "serviceAccountName" not in ok["spec"]
    with pytest.raises(AdmissionError, match="may not reference service accounts"):
        run_chain(FakeServer(), {"metadata": {"name": "m", "annotations": dict(MIRROR)},
                                 "spec": {"serviceAccountName": "default"}})
    with pytest.raises(AdmissionError, match="may not reference secrets"):
        run_chain(FakeServer(), {"metadata": {"name": "m", "annotations": dict(MIRROR)},
                                 "spec": {"volumes": [{"name": "v", "secret": {"secretName": "s"}}]}})


def test_default_account_required_account_and_token():
    srv = FakeServer(serviceaccounts=[sa()])
    pod = run_chain(srv, sapod())
    assert pod["spec"]["serviceAccountName"] == "default"
    with pytest.raises(AdmissionError) as e:
        run_chain(srv, sapod(), {"requireAPIToken": True})
    assert e.value.code == 504 and "No API token found for service account \"default\"" in str(e.value)
    with pytest.raises(AdmissionError, match="error looking up service account myns/default"):
        run_chain(FakeServer(), sapod(), {"requireServiceAccount": True})
    run_chain(FakeServer(), sapod())       # permissive default: admitted


def test_automounts_api_token_and_respects_existing_mount():
    srv = FakeServer(serviceaccounts=[sa(secrets=["token-name"])], secrets=[token("token-name")])
    pod = run_chain(srv, sapod(initContainers=[{"name": "i"}]))
    assert pod["spec"]["volumes"] == [{"name": "token-name", "secret": {"secretName": "token-name", "defaultMode": 0o644}}]
    for c in pod["spec"]["containers"] + pod["spec"]["initContainers"]:
        assert c["volumeMounts"] == [{"name": "token-name", "readOnly": True,
                                      "mountPath": "/var/run/secrets/kubernetes.io/serviceaccount"}]
    own = {"name": "my-mount", "mountPath": "/var/run/secrets/kubernetes.io/serviceaccount"}
    pod = run_chain(srv, sapod(containers=[{"name": "c", "volumeMounts": [dict(own)]}]))
    assert pod["spec"]["containers"][0]["volumeMounts"] == [own]
    assert not pod["spec"].get("volumes")            # no container needed the token volume


def test_image_pull_secrets_added_only_when_pod_has_none():
    srv = FakeServer(serviceaccounts=[sa(pull=["foo", "bar"])])
    pod = run_chain(srv, sapod())
    assert pod["spec"]["imagePullSecrets"] == [{"name": "foo"}, {"name": "bar"}]
    pod = run_chain(srv, sapod(imagePullSecrets=[{"name": "foo"}]))
    assert pod["spec"]["imagePullSecrets"] == [{"name": "foo"}]


def test_enforce_mountable_secrets():
    srv = FakeServer(serviceaccounts=[sa(secrets=["foo"], pull=["foo"], enforce="true")])
    run_chain(srv, sapod(volumes=[{"name": "v", "secret": {"secretName": "foo"}}],
                         containers=[{"name": "c", "env": [{"name": "E", "valueFrom": {"secretKeyRef": {"name": "foo"}}}]}],
                         imagePullSecrets=[{"name": "foo"}]))
    with pytest.raises(AdmissionError, match='volume with secret.secretName="bar" is not allowed because service '
                                             'account default does not reference that secret'):
        run_chain(srv, sapod(volumes=[{"name": "v", "secret": {"secretName": "bar"}}]))
    with pytest.raises(AdmissionError, match="init container i with envVar E referencing secret.secretName=\"bar\""):
        run_chain(srv, sapod(initContainers=[{"name": "i", "env": [{"name": "E",
                                                                     "valueFrom": {"secretKeyRef": {"name": "bar"}}}]}]))
    with pytest.raises(AdmissionError, match="container c with envVar E referencing secret.secretName=\"bar\""):
        run_chain(srv, sapod(containers=[{"name": "c", "env": [{"name": "E",
                                                                "valueFrom": {"secretKeyRef": {"name": "bar"}}}]}]))
    with pytest.raises(AdmissionError, match=r'imagePullSecrets\[0\].name="bar" is not allowed'):
        run_chain(srv, sapod(imagePullSecrets=[{"name": "bar"}]))
    # a permissive account (no annotation, or "false") allows unreferenced secrets
    for enforce in (None, "false"):
        run_chain(FakeServer(serviceaccounts=[sa(enforce=enforce)]),
                  sapod(volumes=[{"name": "v", "secret": {"secretName": "bar"}}], imagePullSecrets=[{"name": "bar"}]))


def test_pod_secret_names_visits_every_reference():
    pod = {"spec": {"imagePullSecrets": [{"name": "pull"}],
                    "initContainers": [{"envFrom": [{"secretRef": {"name": "init-from"}}]}],
                    "containers": [{"env": [{"name": "E", "valueFrom": {"secretKeyRef": {"name": "env"}}}]}],
                    "volumes": [{"secret": {"secretName": "vol"}},
                                {"projected": {"sources": [{"secret": {"name": "proj"}}, {"configMap": {"name": "x"}}]}},
                                {"azureFile": {"secretName": "az"}}, {"rbd": {"secretRef": {"name": "rbd"}}},
                                {"cephfs": {"secretRef": {"name": "ceph"}}}, {"emptyDir": {}}]}}
    assert core.pod_secret_names(pod) == ["pull", "init-from", "env", "vol", "proj", "az", "rbd", "ceph"]
