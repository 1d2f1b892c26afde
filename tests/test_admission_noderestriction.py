"""NodeRestriction admission — port of `plugin/pkg/admission/noderestriction/admission_test.go`
(Test_nodePlugin_Admit: mirror / normal pods bound to self / another node / unbound, for the
pod, pods/status and pods/eviction (named and unnamed) under create / update / delete; pods
referencing a service account, secret, configmap or PVC; own / other node with configSource
rules; unrelated objects and users) plus eviction through the API server."""
import itertools

import pytest

from kubernetes_amd.apiserver.admission import CREATE, DELETE, UPDATE, AdmissionError, Attributes, new_chain
from kubernetes_amd.apiserver.auth import User

NODE = User("system:node:mynode", groups=["system:nodes"])
NOBODY = User("bob", groups=["system:authenticated"])


def pod(name, node, mirror):
    md = {"name": name, "namespace": "ns"}
    if mirror:
        md["annotations"] = {"kubernetes.io/config.mirror": "true"}
    return {"metadata": md, "spec": {"nodeName": node, "containers": [{"name": "c"}]} if node else
            {"containers": [{"name": "c"}]}}


def admit(op, obj, old=None, sub="", user=NODE, resource="pods", name=None):
    chain = new_chain(["NodeRestriction"])
    md = (obj or old or {}).get("metadata") or {}
    a = Attributes(op, resource, sub, md.get("namespace"), md.get("name", "") if name is None else name, obj, old, user)
    chain.admit(a)
    chain.validate(a)


def allowed(*args, **kw):
    try:
        admit(*args, **kw)
        return True
    except AdmissionError:
        return False


def expected(kind, bound, op, sub):
    if sub == "":
        return {CREATE: kind == "mirror" and bound == "self", UPDATE: False, DELETE: bound == "self"}[op]
    if sub == "status":
        return op == UPDATE and bound == "self"
    return op == CREATE and bound == "self"           # eviction


CASES = list(itertools.product(("mirror", "normal"), ("self", "another", "unbound"), (CREATE, UPDATE, DELETE),
                               ("", "status", "eviction")))


@pytest.mark.parametrize("kind,bound,op,sub", CASES, ids=["-".join(c) or "x" for c in CASES])
def test_pod_matrix(kind, bound, op, sub):
    node = {"self": "mynode", "another": "othernode", "unbound": ""}[bound]
    p = pod("p", node, kind == "mirror")
    if sub == "eviction":
        ev = {"metadata": {"name": "p", "namespace": "ns"}}
        got = allowed(op, ev, p, sub)
    else:
        got = allowed(op, p if op != DELETE else None, p, sub)
    assert got == expected(kind, bound, op, sub)
    # the unrelated user is never restricted
    assert allowed(op, p if op != DELETE else None, p, sub, user=NOBODY)


def test_unnamed_eviction_and_unknown_pods():
    p = pod("p", "mynode", False)
    assert allowed(CREATE, {"metadata": {"namespace": "ns"}}, p, "eviction")           # name from the attributes
    assert not allowed(CREATE, {"metadata": {"namespace": "ns"}}, None, "eviction", name="")
    assert not allowed(DELETE, None, None)                                             # unknown pod


@pytest.mark.parametrize("field,value,msg", [
    ("serviceAccountName", "foo", "reference a service account"),
    ("volumes", [{"name": "v", "secret": {"secretName": "s"}}], "reference secrets"),
    ("volumes", [{"name": "v", "configMap": {"name": "c"}}], "reference configmaps"),
    ("volumes", [{"name": "v", "persistentVolumeClaim": {"claimName": "c"}}], "reference persistentvolumeclaims"),
])
def test_mirror_pods_may_not_reference_api_objects(field, value, msg):
    p = pod("p", "mynode", True)
    p["spec"][field] = value
    with pytest.raises(AdmissionError, match=msg):
        admit(CREATE, p)


def node(name, config=None):
    n = {"metadata": {"name": name}, "spec": {}}
    if config is not None:
        n["spec"]["configSource"] = config
    return n


def test_nodes():
    cs1 = {"configMapRef": {"name": "foo", "namespace": "bar", "uid": "fooid"}}
    cs2 = {"configMapRef": {"name": "qux", "namespace": "bar", "uid": "quxid"}}
    assert allowed(CREATE, node("mynode"), resource="nodes")
    assert allowed(CREATE, node("mynode"), resource="nodes", name="")                 # name from the object
    assert allowed(UPDATE, node("mynode"), node("mynode"), resource="nodes")
    assert allowed(DELETE, None, node("mynode"), resource="nodes")
    assert allowed(UPDATE, node("mynode"), node("mynode"), "status", resource="nodes")
    assert not allowed(CREATE, node("mynode", cs1), resource="nodes")
    assert not allowed(UPDATE, node("mynode", cs1), node("mynode"), resource="nodes")
    assert not allowed(UPDATE, node("mynode", cs2), node("mynode", cs1), resource="nodes")
    assert allowed(UPDATE, node("mynode", cs1), node("mynode", cs1), resource="nodes")
    assert allowed(UPDATE, node("mynode"), node("mynode", cs1), resource="nodes")
    for op in (CREATE, UPDATE, DELETE):
        assert not allowed(op, node("othernode") if op != DELETE else None, node("othernode"), resource="nodes")
    assert not allowed(CREATE, node("othernode"), resource="nodes", name="")
    assert not allowed(UPDATE, node("othernode"), node("othernode"), "status", resource="nodes")
    # unrelated objects and users
    svc = {"metadata": {"name": "s", "namespace": "ns"}}
    for op in (CREATE, UPDATE, DELETE):
        assert allowed(op, svc, svc, resource="services")
    assert allowed(UPDATE, node("othernode"), node("othernode"), resource="nodes", user=NOBODY)
    # a node identity without a node name is refused everything
    assert not allowed(CREATE, svc, resource="services", user=User("system:node:", groups=["system:nodes"]))


def test_pvc_status_only():
    old = {"metadata": {"name": "c", "namespace": "ns", "resourceVersion": "1"}, "spec": {}, "status": {}}
    new = dict(old, status={"capacity": {"storage": "2Gi"}})
    assert not allowed(UPDATE, new, old, resource="persistentvolumeclaims")
    assert not allowed(UPDATE, new, old, "status", resource="persistentvolumeclaims")   # gate off
