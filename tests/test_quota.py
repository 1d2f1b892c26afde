"""Resource quota: evaluator usage tables (`pkg/quota/evaluator/core/{pods,services,
persistent_volume_claims}_test.go`), the admission plugin's check-and-charge
(`plugin/pkg/admission/resourcequota/admission_test.go`: below/over limit, constraints, scopes,
status unknown, negative usage, unrelated resources, limitedResources, old objects, conflict
retry), the controller's recount (`resource_quota_controller_test.go` TestSyncResourceQuota) and a
live race: concurrent creates against one quota never overspend it."""
import asyncio
import copy
import time

import pytest

from kubernetes_amd import quota
from kubernetes_amd.api.meta import now_rfc3339
from kubernetes_amd.apiserver.admission import CREATE, DELETE, UPDATE, AdmissionError, Attributes
from kubernetes_amd.apiserver.admission.plugins import ResourceQuota
from kubernetes_amd.client.fake import FakeClient
from kubernetes_amd.client.informer import InformerFactory
from kubernetes_amd.client.rest import APIStatusError
from kubernetes_amd.cluster import LocalCluster
from kubernetes_amd.controllers.misc import ResourceQuotaController


def res(requests=None, limits=None):
    return {"requests": dict(requests or {}), "limits": dict(limits or {})}


def pod(name="p", requests=None, limits=None, init=None, deadline=None, phase=None, ns="test"):
    p = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "namespace": ns},
         "spec": {"containers": [{"name": "c", "image": "i", "resources": res(requests, limits)}]}}
    if init is not None:
        p["spec"]["initContainers"] = [{"name": "i", "image": "i", "resources": init}]
        p["spec"]["containers"] = []
    if deadline is not None:
        p["spec"]["activeDeadlineSeconds"] = deadline
    if phase:
        p["status"] = {"phase": phase}
    return p


def norm(d):
    return {k: str(quota.qty(v)) for k, v in d.items()}


# ------------------------------------------------------------------ evaluator usage tables
POD_USAGE = {
    "init container CPU": (pod(init=res({"cpu": "1m"}, {"cpu": "2m"})),
                           {"requests.cpu": "1m", "limits.cpu": "2m", "pods": "1", "cpu": "1m", "count/pods": "1"}),
    "init container MEM": (pod(init=res({"memory": "1m"}, {"memory": "2m"})),
                           {"requests.memory": "1m", "limits.memory": "2m", "pods": "1", "memory": "1m",
                            "count/pods": "1"}),
    "init container local ephemeral storage": (
        pod(init=res({"ephemeral-storage": "32Mi"}, {"ephemeral-storage": "64Mi"})),
        {"ephemeral-storage": "32Mi", "requests.ephemeral-storage": "32Mi", "limits.ephemeral-storage": "64Mi",
         "pods": "1", "count/pods": "1"}),
    "init container hugepages": (pod(init=res({"hugepages-2Mi": "100Mi"})),
                                 {"hugepages-2Mi": "100Mi", "requests.hugepages-2Mi": "100Mi", "pods": "1",
                                  "count/pods": "1"}),
    "container CPU": (pod(requests={"cpu": "1m"}, limits={"cpu": "2m"}),
                      {"requests.cpu": "1m", "limits.cpu": "2m", "pods": "1", "cpu": "1m", "count/pods": "1"}),
    "terminal pod: only the object count": (pod(requests={"cpu": "1"}, phase="Failed"), {"count/pods": "1"}),
    "extended resource (fork)": (pod(requests={"amd.com/gpu": "2"}, limits={"amd.com/gpu": "2"}),
                                 {"amd.com/gpu": "2", "requests.amd.com/gpu": "2", "pods": "1", "count/pods": "1"}),
}


@pytest.mark.parametrize("name", list(POD_USAGE))
def test_pod_evaluator_usage(name):
    p, want = POD_USAGE[name]
    assert norm(quota.PodEvaluator().usage(p)) == want


def test_pod_past_its_deletion_grace_is_not_charged():
    ev = quota.PodEvaluator()
    p = pod(requests={"cpu": "1"})
    p["metadata"]["deletionGracePeriodSeconds"] = 30
    p["metadata"]["deletionTimestamp"] = now_rfc3339(time.time() - 60)
    assert norm(ev.usage(p)) == {"count/pods": "1"}
    p["metadata"]["deletionTimestamp"] = now_rfc3339(time.time())
    assert norm(ev.usage(p))["cpu"] == "1"


SERVICE_USAGE = {
    "loadbalancer": ({"type": "LoadBalancer", "ports": [{"port": 27443}]},
                     {"services.nodeports": "1", "services.loadbalancers": "1", "services": "1", "count/services": "1"}),
    "loadbalancer_ports": ({"type": "LoadBalancer", "ports": [{"port": 27443}, {"port": 27444}]},
                           {"services.nodeports": "2", "services.loadbalancers": "1", "services": "1",
                            "count/services": "1"}),
    "clusterip": ({"type": "ClusterIP"}, {"services": "1", "services.nodeports": "0", "services.loadbalancers": "0",
                                          "count/services": "1"}),
    "nodeports": ({"type": "NodePort", "ports": [{"port": 27443}]},
                  {"services": "1", "services.nodeports": "1", "services.loadbalancers": "0", "count/services": "1"}),
}


@pytest.mark.parametrize("name", list(SERVICE_USAGE))
def test_service_evaluator_usage(name):
    spec, want = SERVICE_USAGE[name]
    assert norm(quota.ServiceEvaluator().usage({"spec": spec})) == want


def test_pvc_evaluator_usage_by_storage_class():
    pvc = {"spec": {"storageClassName": "gold", "resources": {"requests": {"storage": "10Gi"}}}}
    assert norm(quota.PVCEvaluator().usage(pvc)) == {
        "persistentvolumeclaims": "1", "count/persistentvolumeclaims": "1", "requests.storage": "10Gi",
        "gold.storageclass.storage.k8s.io/persistentvolumeclaims": "1",
        "gold.storageclass.storage.k8s.io/requests.storage": "10Gi"}
    assert quota.PVCEvaluator().matching_resources(["gold.storageclass.storage.k8s.io/requests.storage", "cpu"]) == \
        ["gold.storageclass.storage.k8s.io/requests.storage"]


def test_pod_constraints_require_explicit_cpu_and_memory():
    ev = quota.PodEvaluator()
    assert ev.constraints(["cpu"], pod(requests={"memory": "1Gi"})) == "must specify cpu"
    assert ev.constraints(["cpu", "memory"], pod(requests={"cpu": "1", "memory": "1Gi"})) is None
    assert ev.constraints(["pods"], pod()) is None


def test_object_count_names():
    assert quota.object_count_name("pods") == "count/pods"
    assert quota.object_count_name("deployments", "apps") == "count/deployments.apps"
    reg = quota.Registry()
    assert reg.get("", "configmaps").matching_resources(["configmaps", "count/configmaps", "secrets"]) == \
        ["configmaps", "count/configmaps"]
    assert reg.for_name("count/widgets.example.com").resource == "widgets"


# ------------------------------------------------------------------ admission
class FakeServer:
    """What the plugin needs from the API server: the namespace's quotas and a CAS status
    write (409 when the resourceVersion moved)."""

    def __init__(self, *quotas):
        self.quotas = {q["metadata"]["name"]: copy.deepcopy(q) for q in quotas}
        self.writes = []
        self.interfere = None      # callable run before a write: simulates a concurrent writer

    async def quota_objects(self, namespace, fresh=False):
        return [copy.deepcopy(q) for q in self.quotas.values() if q["metadata"].get("namespace") == namespace]

    async def write_quota_status(self, q):
        if self.interfere:
            f, self.interfere = self.interfere, None
            f(self.quotas)
        cur = self.quotas[q["metadata"]["name"]]
        if q["metadata"].get("resourceVersion") != cur["metadata"].get("resourceVersion"):
            raise APIStatusError(409, {"message": "conflict"})
        q = copy.deepcopy(q)
        q["metadata"]["resourceVersion"] = str(int(cur["metadata"]["resourceVersion"]) + 1)
        self.quotas[q["metadata"]["name"]] = q
        self.writes.append(q)


def rq(name="quota", hard=None, used=None, scopes=None, ns="test"):
    q = {"metadata": {"name": name, "namespace": ns, "resourceVersion": "124"},
         "spec": {"hard": dict(hard or {})}, "status": {"hard": dict(hard or {})}}
    if used is not None:
        q["status"]["used"] = dict(used)
    if scopes:
        q["spec"]["scopes"] = list(scopes)
    return q


def admit(server, obj, op=CREATE, resource="pods", old=None, sub="", config=None):
    plugin = ResourceQuota(server, config)
    a = Attributes(op, resource, sub, obj["metadata"].get("namespace", "test"), obj["metadata"]["name"], obj, old)
    if not plugin.handles(op):
        return
    asyncio.run(plugin.charge(a))


BASE = dict(hard={"cpu": "3", "memory": "100Gi", "pods": "5"}, used={"cpu": "1", "memory": "50Gi", "pods": "3"})


def test_admit_below_quota_limit():
    s = FakeServer(rq(**BASE))
    admit(s, pod("allowed-pod", requests={"cpu": "100m", "memory": "2Gi"}))
    assert len(s.writes) == 1
    assert norm(s.writes[-1]["status"]["used"]) == {"cpu": "1100m", "memory": "52Gi", "pods": "4"}


def test_admit_exceed_quota_limit():
    s = FakeServer(rq(**BASE))
    with pytest.raises(AdmissionError) as ei:
        admit(s, pod("not-allowed-pod", requests={"cpu": "3", "memory": "2Gi"}))
    assert str(ei.value) == "exceeded quota: quota, requested: cpu=3, used: cpu=1, limited: cpu=3"
    assert not s.writes


def test_admit_enforce_quota_constraints():
    s = FakeServer(rq(hard={"cpu": "3", "memory": "100Gi", "limits.memory": "200Gi", "pods": "5"},
                      used={"cpu": "1", "memory": "50Gi", "limits.memory": "100Gi", "pods": "3"}))
    with pytest.raises(AdmissionError) as ei:
        admit(s, pod("not-allowed-pod", requests={"cpu": "100m", "memory": "2Gi"}, limits={"cpu": "200m"}))
    assert "must specify limits.memory" in str(ei.value)


def test_admit_pod_in_namespace_without_quota():
    s = FakeServer(rq(ns="other", **BASE))
    admit(s, pod("p", requests={"cpu": "100m"}))
    assert not s.writes


def test_admit_below_terminating_quota_limit():
    s = FakeServer(rq("quota-non-terminating", scopes=["NotTerminating"], **BASE),
                   rq("quota-terminating", scopes=["Terminating"], **BASE))
    admit(s, pod("allowed-pod", requests={"cpu": "100m", "memory": "2Gi"}, deadline=30))
    assert [w["metadata"]["name"] for w in s.writes] == ["quota-terminating"]
    assert norm(s.writes[0]["status"]["used"]) == {"cpu": "1100m", "memory": "52Gi", "pods": "4"}


def test_admit_below_best_effort_quota_limit():
    s = FakeServer(rq("quota-besteffort", hard={"pods": "5"}, used={"pods": "3"}, scopes=["BestEffort"]),
                   rq("quota-not-besteffort", hard={"pods": "5"}, used={"pods": "3"}, scopes=["NotBestEffort"]))
    admit(s, pod("allowed-pod"))
    assert [w["metadata"]["name"] for w in s.writes] == ["quota-besteffort"]
    s = FakeServer(rq("quota-besteffort", hard={"pods": "5"}, used={"pods": "3"}, scopes=["BestEffort"]))
    admit(s, pod("burstable", requests={"cpu": "100m"}))          # Burstable: the BestEffort quota ignores it
    assert not s.writes


def test_status_unknown_is_refused():
    s = FakeServer(rq(hard={"pods": "5"}))
    with pytest.raises(AdmissionError) as ei:
        admit(s, pod("p"))
    assert str(ei.value) == "status unknown for quota: quota"


def test_admit_rejects_negative_usage():
    s = FakeServer(rq(hard={"cpu": "3", "pods": "5"}, used={"cpu": "1", "pods": "3"}))
    with pytest.raises(AdmissionError) as ei:
        admit(s, pod("bad", requests={"cpu": "-1"}))
    assert "quota usage is negative for resource(s): cpu" in str(ei.value)


def test_admit_when_unrelated_resource_exceeds_quota():
    s = FakeServer(rq(hard={"services": "3", "pods": "4"}, used={"services": "4", "pods": "1"}))
    admit(s, pod("allowed"))
    assert norm(s.writes[-1]["status"]["used"]) == {"services": "4", "pods": "2"}


LIMITED = {"limitedResources": [{"resource": "pods", "matchContains": ["requests.cpu"]}]}


def test_limited_resource_needs_a_covering_quota():
    with pytest.raises(AdmissionError) as ei:
        admit(FakeServer(), pod("p", requests={"cpu": "1"}), config=LIMITED)
    assert str(ei.value) == "insufficient quota to consume: requests.cpu"
    admit(FakeServer(), pod("p", requests={"memory": "1Gi"}), config=LIMITED)      # not a matching resource
    s = FakeServer(rq(hard={"requests.cpu": "4"}, used={"requests.cpu": "1"}))
    admit(s, pod("p", requests={"cpu": "1"}), config=LIMITED)
    assert norm(s.writes[-1]["status"]["used"]) == {"requests.cpu": "2"}
    with pytest.raises(AdmissionError):       # a quota that does not cover requests.cpu does not count
        admit(FakeServer(rq(hard={"memory": "4Gi"}, used={"memory": "0"})), pod("p", requests={"cpu": "1"}),
              config=LIMITED)


def test_service_update_is_charged_the_delta():
    old = {"metadata": {"name": "svc", "namespace": "test", "resourceVersion": "1"}, "spec": {"type": "ClusterIP",
                                                                                              "ports": [{"port": 80}]}}
    new = copy.deepcopy(old)
    new["spec"] = {"type": "NodePort", "ports": [{"port": 80}, {"port": 81}]}
    s = FakeServer(rq(hard={"services": "10", "services.nodeports": "10"}, used={"services": "1",
                                                                                "services.nodeports": "0"}))
    admit(s, new, UPDATE, "services", old)
    assert norm(s.writes[-1]["status"]["used"]) == {"services": "1", "services.nodeports": "2"}
    # "create on update" (no resourceVersion on the old object): the full usage is charged
    s = FakeServer(rq(hard={"services": "10"}, used={"services": "1"}))
    old2 = copy.deepcopy(old)
    del old2["metadata"]["resourceVersion"]
    admit(s, new, UPDATE, "services", old2)
    assert norm(s.writes[-1]["status"]["used"]) == {"services": "2"}


def test_deletes_and_subresources_are_ignored():
    s = FakeServer(rq(hard={"pods": "0"}, used={"pods": "0"}))
    admit(s, pod("p"), DELETE)
    admit(s, pod("p"), sub="status")
    assert not s.writes


def test_conflicting_writer_is_rechecked_against_the_fresh_quota():
    s = FakeServer(rq(hard={"pods": "2"}, used={"pods": "0"}))

    def other(quotas):                  # another request charged the quota first
        q = quotas["quota"]
        q["status"]["used"] = {"pods": "1"}
        q["metadata"]["resourceVersion"] = "125"
    s.interfere = other
    admit(s, pod("a"))
    assert norm(s.quotas["quota"]["status"]["used"]) == {"pods": "2"}
    with pytest.raises(AdmissionError):
        admit(s, pod("b"))


# ------------------------------------------------------------------ controller
def _sync(*objs):
    async def main():
        c = FakeClient(*objs)
        f = InformerFactory(c)
        qc = ResourceQuotaController(c, f)
        qc.setup()
        f.start()
        await f.wait_for_cache_sync()
        await qc.sync("testing/quota")
        writes = [a for a in c.actions if a.verb in ("update", "patch") and a.resource == "resourcequotas"]
        return (await c.get("resourcequotas", "quota", "testing")).get("status") or {}, writes
    return asyncio.run(main())


def _controller_quota(hard, status=None):
    q = {"apiVersion": "v1", "kind": "ResourceQuota", "metadata": {"name": "quota", "namespace": "testing"},
         "spec": {"hard": dict(hard)}}
    if status is not None:
        q["status"] = status
    return q


def test_sync_resource_quota_counts_live_pods():
    pods = [pod("pod-running", requests={"cpu": "100m", "memory": "1Gi"}, phase="Running", ns="testing"),
            pod("pod-running-2", requests={"cpu": "100m", "memory": "1Gi"}, phase="Running", ns="testing"),
            pod("pod-failed", requests={"cpu": "100m", "memory": "1Gi"}, phase="Failed", ns="testing")]
    st, writes = _sync(_controller_quota({"cpu": "3", "memory": "100Gi", "pods": "5"}), *pods)
    assert writes and norm(st["used"]) == {"cpu": "200m", "memory": "2Gi", "pods": "2"}
    assert norm(st["hard"]) == {"cpu": "3", "memory": "100Gi", "pods": "5"}


def test_sync_resource_quota_spec_hard_updated():
    st, writes = _sync(_controller_quota({"cpu": "4"}, {"hard": {"cpu": "3"}, "used": {"cpu": "0"}}))
    assert writes and norm(st["hard"]) == {"cpu": "4"} and norm(st["used"]) == {"cpu": "0"}


def test_sync_resource_quota_unchanged_writes_nothing():
    st, writes = _sync(_controller_quota({"cpu": "4"}, {"hard": {"cpu": "4"}, "used": {"cpu": "0"}}))
    assert not writes


def test_sync_counts_objects_and_scopes():
    objs = [{"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": f"cm{i}", "namespace": "testing"}}
            for i in range(3)]
    objs += [pod("t", deadline=10, ns="testing"), pod("nt", ns="testing")]
    st, _ = _sync(_controller_quota({"configmaps": "10", "count/configmaps": "10", "pods": "9"}), *objs)
    assert norm(st["used"]) == {"configmaps": "3", "count/configmaps": "3", "pods": "2"}
    q = _controller_quota({"pods": "9"})
    q["spec"]["scopes"] = ["Terminating"]
    st, _ = _sync(q, *objs)
    assert norm(st["used"]) == {"pods": "1"}


# ------------------------------------------------------------------ live
def test_concurrent_creates_never_overspend_a_quota(run):
    async def main():
        async with LocalCluster(nodes=1, gpus_per_node=1, controllers=["resourcequota"]) as cl:
            c = cl.client
            await c.create("resourcequotas", {"metadata": {"name": "q", "namespace": "default"},
                                              "spec": {"hard": {"pods": "2", "count/configmaps": "1"}}})

            async def counted():
                st = (await c.get("resourcequotas", "q", "default")).get("status") or {}
                return (st.get("used") or {}).get("pods") == "0"
            await cl.wait_for(counted, timeout=30)
            res = await asyncio.gather(*[c.create("pods", {"metadata": {"name": f"r{i}", "namespace": "default"},
                                                           "spec": {"containers": [{"name": "c", "image": "x"}]}})
                                         for i in range(5)], return_exceptions=True)
            ok = [r for r in res if not isinstance(r, Exception)]
            errs = [r for r in res if isinstance(r, Exception)]
            assert len(ok) == 2 and all(isinstance(e, APIStatusError) and e.code in (403, 409) for e in errs), res
            await c.create("configmaps", {"metadata": {"name": "a", "namespace": "default"}})
            with pytest.raises(APIStatusError) as ei:
                await c.create("configmaps", {"metadata": {"name": "b", "namespace": "default"}})
            assert ei.value.code == 403 and "count/configmaps" in ei.value.status["message"]
            # replenishment: deleting a pod frees its slot once the controller recounts
            await c.delete("pods", ok[0]["metadata"]["name"], "default", grace_period=0)

            async def freed():
                st = (await c.get("resourcequotas", "q", "default")).get("status") or {}
                return (st.get("used") or {}).get("pods") == "1"
            await cl.wait_for(freed, timeout=30)
            await c.create("pods", {"metadata": {"name": "late", "namespace": "default"},
                                    "spec": {"containers": [{"name": "c", "image": "x"}]}})
    run(main(), timeout=90)


def test_quota_validation():
    """ValidateResourceQuota: standard / qualified names, scopes that can track every hard name,
    immutable scopes."""
    from kubernetes_amd.api.validation_ext import validate_resource_quota, validate_update

    def errs(hard, scopes=None):
        o = {"metadata": {"name": "q", "namespace": "d"}, "spec": {"hard": hard}}
        if scopes:
            o["spec"]["scopes"] = scopes
        return [str(e) for e in validate_resource_quota(o)]
    assert errs({"pods": "1", "count/deployments.apps": "2", "requests.amd.com/gpu": "4",
                 "gold.storageclass.storage.k8s.io/requests.storage": "1Gi", "hugepages-2Mi": "1Gi"}) == []
    assert errs({"foo": "1"}) and errs({"pods": "-1"})
    assert any("unsupported scope" in e for e in errs({"cpu": "1"}, ["BestEffort"]))
    assert any("unsupported scope" in e for e in errs({"services": "1"}, ["Terminating"]))
    assert errs({"pods": "1", "cpu": "1"}, ["NotBestEffort"]) == []
    old = {"metadata": {"name": "q", "namespace": "d", "uid": "u", "resourceVersion": "1"},
           "spec": {"hard": {"pods": "1"}, "scopes": ["Terminating"]}}
    new = dict(old, spec={"hard": {"pods": "1"}, "scopes": ["NotTerminating"]})
    assert any("immutable" in str(e) for e in validate_update("ResourceQuota", new, old))
