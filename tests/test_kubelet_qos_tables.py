"""QoS class and OOM score tables ported from `pkg/apis/core/v1/helper/qos/qos_test.go`
(TestGetPodQOS) and `pkg/kubelet/qos/policy_test.go` (TestGetContainerOOMScoreAdjust).
GPU limits use the fork's resource name and amd.com/gpu alike; neither affects the class."""
import pytest

from kubernetes_amd.apiserver.registry import qos_class
from kubernetes_amd.kubelet.qos import oom_score_adj


def rl(cpu="", memory="", **extra):
    r = {}
    if cpu:
        r["cpu"] = cpu
    if memory:
        r["memory"] = memory
    r.update({k.replace("_", "-").replace("--", "/"): v for k, v in extra.items()})
    return r


def ctr(req, lim):
    return {"name": "c", "resources": {"requests": req, "limits": lim}}


def pod(*containers):
    return {"metadata": {"name": "p"}, "spec": {"containers": list(containers)}}


GPU = {"alpha.kubernetes.io/nvidia-gpu": "2"}
AMD = {"amd.com/gpu": "2"}

QOS_CASES = [
    ("guaranteed", pod(ctr(rl("100m", "100Mi"), rl("100m", "100Mi"))), "Guaranteed"),
    ("guaranteed-with-gpu", pod(ctr(rl("100m", "100Mi"), {**rl("100m", "100Mi"), **GPU})), "Guaranteed"),
    ("guaranteed-with-amd-gpu", pod(ctr(rl("100m", "100Mi"), {**rl("100m", "100Mi"), **AMD})), "Guaranteed"),
    ("guaranteed-guaranteed", pod(ctr(rl("100m", "100Mi"), rl("100m", "100Mi")),
                                  ctr(rl("100m", "100Mi"), rl("100m", "100Mi"))), "Guaranteed"),
    ("guaranteed-guaranteed-with-gpu", pod(ctr(rl("100m", "100Mi"), {**rl("100m", "100Mi"), **GPU}),
                                           ctr(rl("100m", "100Mi"), rl("100m", "100Mi"))), "Guaranteed"),
    ("best-effort-best-effort", pod(ctr({}, {}), ctr({}, {})), "BestEffort"),
    ("best-effort-best-effort-with-gpu", pod(ctr({}, dict(GPU)), ctr({}, {})), "BestEffort"),
    ("best-effort-with-gpu", pod(ctr({}, dict(GPU))), "BestEffort"),
    ("best-effort-burstable", pod(ctr({}, dict(GPU)), ctr(rl("1"), rl("2"))), "Burstable"),
    ("best-effort-guaranteed", pod(ctr({}, dict(GPU)), ctr(rl("10m", "100Mi"), rl("10m", "100Mi"))), "Burstable"),
    ("burstable-cpu-guaranteed-memory", pod(ctr(rl("", "100Mi"), rl("", "100Mi"))), "Burstable"),
    ("burstable-no-limits", pod(ctr(rl("100m", "100Mi"), {})), "Burstable"),
    ("burstable-guaranteed", pod(ctr(rl("1", "100Mi"), rl("2", "100Mi")),
                                 ctr(rl("100m", "100Mi"), rl("100m", "100Mi"))), "Burstable"),
    ("burstable-unbounded-but-requests-match-limits", pod(ctr(rl("100m", "100Mi"), rl("200m", "200Mi")),
                                                          ctr(rl("100m", "100Mi"), {})), "Burstable"),
    ("burstable-1", pod(ctr(rl("10m", "100Mi"), rl("100m", "200Mi"))), "Burstable"),
    ("burstable-2", pod(ctr(rl("0", "0"), {**rl("100m", "200Mi"), **GPU})), "Burstable"),
    ("burstable-hugepages", pod(ctr({**rl("0", "0"), "hugepages-2Mi": "1Gi"},
                                    {**rl("0", "0"), "hugepages-2Mi": "1Gi"})), "Burstable"),
    # summed, not per container: equal totals with unequal containers are still Guaranteed
    ("sums-match", pod(ctr(rl("100m", "100Mi"), rl("200m", "50Mi")), ctr(rl("200m", "50Mi"), rl("100m", "100Mi"))),
     "Guaranteed"),
    # undefaulted pod with limits only: no requests to match
    ("limits-only-undefaulted", pod(ctr({}, rl("1", "1Gi"))), "Burstable"),
    ("equal-quantities-different-spelling", pod(ctr(rl("1", "1024Mi"), rl("1000m", "1Gi"))), "Guaranteed"),
]


@pytest.mark.parametrize("name,p,want", QOS_CASES, ids=[c[0] for c in QOS_CASES])
def test_get_pod_qos(name, p, want):
    assert qos_class(p) == want


STANDARD = 8_000_000_000

OOM_CASES = [
    ("cpu-limit", pod(ctr({}, rl("10"))), 4_000_000_000, 999, 999),
    ("memory-limit-cpu-request", pod(ctr(rl("0"), rl("", "10G"))), 8_000_000_000, 999, 999),
    ("zero-memory-limit", pod(ctr({}, rl("", "0"))), 7_230_457_451, 1000, 1000),
    ("no-request-limit", pod(ctr({}, {})), 4_000_000_000, 1000, 1000),
    ("equal-request-limit", pod(ctr(rl("5m", "10G"), rl("5m", "10G"))), 123_456_789, -998, -998),
    ("cpu-unlimited-memory-limited-with-requests", pod(ctr(rl("5m", str(STANDARD // 2)), rl("", "10G"))),
     STANDARD, 495, 505),
    ("request-no-limit", pod(ctr(rl("5m", str(STANDARD - 1)), {})), STANDARD, 2, 2),
]


@pytest.mark.parametrize("name,p,cap,lo,hi", OOM_CASES, ids=[c[0] for c in OOM_CASES])
def test_get_container_oom_score_adjust(name, p, cap, lo, hi):
    adj = oom_score_adj(p, p["spec"]["containers"][0], cap)
    assert lo <= adj <= hi, adj


def test_hugepages_limit_makes_pod_burstable():
    """Reference quirk: qosLimitsFound counts hugepages, compared against the 2 cpu/memory names."""
    p = pod(ctr({**rl("1", "1Gi"), "hugepages-2Mi": "2Mi"}, {**rl("1", "1Gi"), "hugepages-2Mi": "2Mi"}))
    assert qos_class(p) == "Burstable"


# -- pkg/kubelet/types/pod_update_test.go TestIsCriticalPod ---------------------------------------
@pytest.mark.parametrize("ns,value,want", [("ns", "", False), ("ns", "abc", False), ("kube-system", "abc", False),
                                          ("kube-system", "", True)])
def test_is_critical_pod(ns, value, want):
    from kubernetes_amd.kubelet.qos import CRITICAL_POD_ANNOTATION, is_critical_pod
    pod = {"metadata": {"name": "p", "namespace": ns, "annotations": {CRITICAL_POD_ANNOTATION: value}}, "spec": {}}
    assert is_critical_pod(pod) is want
