"""Scheduler predicates against the reference tables (`plugin/pkg/scheduler/algorithm/
predicates/predicates_test.go` TestPodFitsResources incl. init containers and extended
resources, TestPodFitsHostPorts incl. the 0.0.0.0 wildcard, TestPodFitsHost) and the FitError
message that lists every insufficient resource."""
import pytest

from kubernetes_amd.scheduler import predicates as P
from kubernetes_amd.scheduler.cache import NodeInfo, PodInfo
from kubernetes_amd.scheduler.generic import FitError

EXT = "example.com/aaa"


def node(cpu=10, mem=20, pods=32, ext=5):
    return {"metadata": {"name": "m1", "labels": {}}, "spec": {},
            "status": {"allocatable": {"cpu": f"{cpu}m", "memory": str(mem), "pods": str(pods), EXT: str(ext)},
                       "conditions": [{"type": "Ready", "status": "True"}]}}


def res(cpu=0, mem=0, ext=0):
    r = {}
    if cpu:
        r["cpu"] = f"{cpu}m"
    if mem:
        r["memory"] = str(mem)
    if ext:
        r[EXT] = str(ext)
    return {"requests": r, "limits": {EXT: str(ext)} if ext else {}}


def pod(*usage, init=(), node_name=""):
    spec = {"containers": [{"name": f"c{i}", "resources": res(*u)} for i, u in enumerate(usage)]}
    if init:
        spec["initContainers"] = [{"name": f"i{i}", "resources": res(*u)} for i, u in enumerate(init)]
    if node_name:
        spec["nodeName"] = node_name
    return {"metadata": {"name": "p", "namespace": "default", "uid": "p"}, "spec": spec}


def fits(the_pod, existing, **alloc):
    ni = NodeInfo()
    ni.set_node(node(**alloc))
    for i, e in enumerate(existing):
        ni.add_pod(f"e{i}", e, PodInfo(e))
    return P.pod_fits_resources(the_pod, PodInfo(the_pod), ni, None)


@pytest.mark.parametrize("the_pod,existing,expect", [
    (pod(), [pod((10, 20))], None),                                             # no resources requested always fits
    (pod((1, 1)), [pod((10, 20))], ("Insufficient cpu", "Insufficient memory")),   # too many resources fails
    (pod((1, 1), init=[(3, 1)]), [pod((8, 19))], "Insufficient cpu"),             # init container cpu
    (pod((1, 1), init=[(3, 1), (2, 1)]), [pod((8, 19))], "Insufficient cpu"),     # highest init container cpu
    (pod((1, 1), init=[(1, 3)]), [pod((9, 19))], "Insufficient memory"),
    (pod((1, 1), init=[(1, 1)]), [pod((9, 19))], None),                         # max, not sum
    (pod((1, 1), init=[(1, 1), (1, 1)]), [pod((9, 19))], None),
    (pod((1, 1)), [pod((5, 5))], None),                                         # both resources fit
    (pod((2, 1)), [pod((9, 5))], "Insufficient cpu"),
    (pod((1, 2)), [pod((5, 19))], "Insufficient memory"),
    (pod((5, 1)), [pod((5, 19))], None),                                        # equal edge case
    (pod((4, 1), init=[(5, 1)]), [pod((5, 19))], None),                         # equal edge case, init container
    (pod((0, 0, 1)), [pod()], None),                                            # extended resource fits
    (pod((0, 0, 10)), [pod()], f"Insufficient {EXT}"),
    (pod((0, 0, 1)), [pod((0, 0, 5))], f"Insufficient {EXT}"),
    (pod(init=[(0, 0, 6)]), [pod()], f"Insufficient {EXT}"),
])
def test_pod_fits_resources(the_pod, existing, expect):
    assert fits(the_pod, existing) == expect


def test_pod_count_limit():
    assert fits(pod((1, 1)), [pod((10, 20))], pods=1) == "Insufficient pods"


def test_fit_error_counts_every_reason():
    e = FitError(pod(), 2, {"m1": ("Insufficient cpu", "Insufficient memory"), "m2": "Insufficient cpu"})
    assert str(e) == "0/2 nodes are available: 2 Insufficient cpu, 1 Insufficient memory."


def port_pod(*specs):
    ports = []
    for s in specs:
        proto, ip, port = s.split("/")
        ports.append({"protocol": proto, "hostIP": ip, "hostPort": int(port), "containerPort": int(port)})
    return {"metadata": {"name": "pp", "namespace": "default"}, "spec": {"containers": [{"name": "c", "ports": ports}]}}


@pytest.mark.parametrize("want,have,ok", [
    ((), (), True),
    (("UDP/127.0.0.1/8080",), ("UDP/127.0.0.1/9090",), True),
    (("UDP/127.0.0.1/8080",), ("UDP/127.0.0.1/8080",), False),
    (("TCP/127.0.0.1/8080",), ("TCP/127.0.0.1/8080",), False),
    (("TCP/127.0.0.1/8080",), ("TCP/127.0.0.2/8080",), True),
    (("UDP/127.0.0.1/8080",), ("TCP/127.0.0.1/8080",), True),
    (("UDP/127.0.0.1/8000", "UDP/127.0.0.1/8080"), ("UDP/127.0.0.1/8080",), False),
    (("TCP/127.0.0.1/8001", "UDP/127.0.0.1/8080"), ("TCP/127.0.0.1/8001", "UDP/127.0.0.1/8081"), False),
    (("TCP/0.0.0.0/8001",), ("TCP/127.0.0.1/8001",), False),
    (("TCP/10.0.10.10/8001", "TCP/0.0.0.0/8001"), ("TCP/127.0.0.1/8001",), False),
    (("TCP/127.0.0.1/8001",), ("TCP/0.0.0.0/8001",), False),
    (("UDP/127.0.0.1/8001",), ("TCP/0.0.0.0/8001",), True),
    (("UDP/127.0.0.1/8001",), ("TCP/0.0.0.0/8001", "UDP/0.0.0.0/8001"), False),
])
def test_pod_fits_host_ports(want, have, ok):
    ni = NodeInfo()
    ni.set_node(node())
    existing = port_pod(*have)
    ni.add_pod("e", existing, PodInfo(existing))
    p = port_pod(*want)
    assert (P.pod_fits_host_ports(p, PodInfo(p), ni, None) is None) == ok


@pytest.mark.parametrize("node_name,ok", [("", True), ("m1", True), ("m2", False)])
def test_pod_fits_host(node_name, ok):
    ni = NodeInfo()
    ni.set_node(node())
    p = pod(node_name=node_name)
    assert (P.pod_fits_host(p, PodInfo(p), ni, None) is None) == ok
