"""PodDisruptionBudgets: the disruption controller's status computation
(`pkg/controller/disruption/disruption_test.go` — TestNoSelector, TestUnavailable,
TestIntegerMaxUnavailable(WithScaling), TestNakedPod, TestReplicaSet, TestReplicationController,
TestStatefulSetController, TestMultipleControllers, TestUpdateDisruptedPods) over the fake client,
and the eviction subresource's check-and-decrement
(`pkg/registry/core/pod/storage/eviction.go`) against a live API server."""
import asyncio

import pytest

from kubernetes_amd.api.meta import now_rfc3339
from kubernetes_amd.client.fake import FakeClient
from kubernetes_amd.client.informer import InformerFactory
from kubernetes_amd.client.rest import APIStatusError
from kubernetes_amd.cluster import LocalCluster
from kubernetes_amd.controllers.misc import DisruptionController

LABELS = {"foo": "bar"}


def pdb(min_available=None, max_unavailable=None, selector=None, status=None):
    spec = {"selector": {"matchLabels": dict(LABELS)} if selector is None else selector}
    if min_available is not None:
        spec["minAvailable"] = min_available
    if max_unavailable is not None:
        spec["maxUnavailable"] = max_unavailable
    o = {"apiVersion": "policy/v1beta1", "kind": "PodDisruptionBudget",
         "metadata": {"name": "pdb", "namespace": "default", "uid": "pdb-uid", "generation": 1}, "spec": spec}
    if status:
        o["status"] = status
    return o


def pod(name, ready=True, owner=None, deleting=False):
    p = {"apiVersion": "v1", "kind": "Pod",
         "metadata": {"name": name, "namespace": "default", "uid": f"{name}-uid", "labels": dict(LABELS)},
         "spec": {}, "status": {"conditions": [{"type": "Ready", "status": "True"}] if ready else []}}
    if owner is not None:
        p["metadata"]["ownerReferences"] = [{"apiVersion": owner["apiVersion"], "kind": owner["kind"],
                                             "name": owner["metadata"]["name"], "uid": owner["metadata"]["uid"],
                                             "controller": True}]
    if deleting:
        p["metadata"]["deletionTimestamp"] = now_rfc3339()
    return p


def ctl(kind, name, replicas, owner=None):
    api = {"ReplicationController": "v1"}.get(kind, "apps/v1")
    o = {"apiVersion": api, "kind": kind, "metadata": {"name": name, "namespace": "default", "uid": f"{name}-uid"},
         "spec": {"replicas": replicas, "selector": {"matchLabels": dict(LABELS)} if kind != "ReplicationController"
                  else dict(LABELS)}}
    if owner is not None:
        o["metadata"]["ownerReferences"] = [{"apiVersion": "apps/v1", "kind": owner["kind"], "name": owner["metadata"]["name"],
                                             "uid": owner["metadata"]["uid"], "controller": True}]
    return o


def status_of(*objs):
    """One sync of the budget over `objs`; returns (allowed, currentHealthy, desiredHealthy,
    expectedPods, disruptedPods names)."""
    async def main():
        c = FakeClient(*objs)
        f = InformerFactory(c)
        dc = DisruptionController(c, f)
        dc.setup()
        f.start()
        await f.wait_for_cache_sync()
        await dc.sync("default/pdb")
        return (await c.get("poddisruptionbudgets", "pdb", "default")).get("status") or {}
    st = asyncio.run(main())
    return (st.get("disruptionsAllowed"), st.get("currentHealthy"), st.get("desiredHealthy"), st.get("expectedPods"),
            sorted(st.get("disruptedPods") or ()))


def test_no_selector_selects_nothing():
    assert status_of(pdb(min_available=3, selector={}), pod("yo"))[:4] == (0, 0, 3, 0)


def test_unavailable_counts():
    pods = [pod(f"p{i}") for i in range(4)]
    for i in range(4):
        assert status_of(pdb(min_available=3), *pods[:i])[:4] == (0, i, 3, i)
    assert status_of(pdb(min_available=3), *pods)[:4] == (1, 4, 3, 4)
    pods[0] = pod("p0", ready=False)
    assert status_of(pdb(min_available=3), *pods)[:4] == (0, 3, 3, 4)


def test_integer_max_unavailable_needs_a_controller():
    assert status_of(pdb(max_unavailable=1))[0] == 0
    assert status_of(pdb(max_unavailable=1), pod("naked"))[0] == 0


def test_integer_max_unavailable_follows_the_controller_scale():
    rs = ctl("ReplicaSet", "rs", 7)
    assert status_of(pdb(max_unavailable=2), rs, pod("p", owner=rs))[:4] == (0, 1, 5, 7)
    rs = ctl("ReplicaSet", "rs", 5)
    assert status_of(pdb(max_unavailable=2), rs, pod("p", owner=rs))[:4] == (0, 1, 3, 5)


def test_naked_pod_with_a_percentage():
    assert status_of(pdb(min_available="28%"))[0] == 0
    assert status_of(pdb(min_available="28%"), pod("naked"))[0] == 0


def test_replica_set_without_deployment():
    rs = ctl("ReplicaSet", "rs", 10)
    assert status_of(pdb(min_available="20%"), rs, pod("p", owner=rs))[:4] == (0, 1, 2, 10)


@pytest.mark.parametrize("kind", ["ReplicationController", "StatefulSet"])
def test_controller_scale_with_a_percentage(kind):
    """TestReplicationController / TestStatefulSetController: 3 replicas, 34% -> 2 desired; the
    third ready pod allows one disruption."""
    c = ctl(kind, "c", 3)
    pods = [pod(f"p{i}", owner=c) for i in range(3)]
    for i in range(3):
        exp = (1, 3, 2, 3) if i == 2 else (0, i + 1, 2, 3)
        assert status_of(pdb(min_available="34%"), c, *pods[:i + 1])[:4] == exp


def test_deployment_scale_through_its_replica_set():
    d = ctl("Deployment", "d", 4)
    rs = ctl("ReplicaSet", "rs", 4, owner=d)
    pods = [pod(f"p{i}", owner=rs) for i in range(4)]
    assert status_of(pdb(min_available="50%"), d, rs, *pods)[:4] == (2, 4, 2, 4)


def test_multiple_controllers_sum_their_scale():
    """TestMultipleControllers: pods of two controllers count both scales (1 + 1 replicas here);
    a naked pod among them makes the count unknowable -> no disruption."""
    a, b = ctl("ReplicationController", "a", 1), ctl("ReplicationController", "b", 1)
    assert status_of(pdb(min_available="1%"), a, b, pod("pa", owner=a), pod("pb", owner=b))[:4] == (1, 2, 1, 2)
    assert status_of(pdb(min_available="1%"), a, b, pod("pa", owner=a), pod("pb", owner=b), pod("naked"))[0] == 0


def test_update_disrupted_pods():
    now = now_rfc3339()
    import time
    old = now_rfc3339(time.time() - 300)
    st = {"disruptedPods": {"p1": now, "p2": old, "p3": now, "notthere": now}}
    got = status_of(pdb(min_available=1, status=st), pod("p1", deleting=True), pod("p2"), pod("p3"))
    assert got == (0, 1, 1, 3, ["p3"])


def _pdb_obj(name, min_available):
    return {"apiVersion": "policy/v1beta1", "kind": "PodDisruptionBudget",
            "metadata": {"name": name, "namespace": "default"},
            "spec": {"minAvailable": min_available, "selector": {"matchLabels": {"app": "web"}}}}


def _bare_pod(name):
    return {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "namespace": "default", "labels": {"app": "web"}},
            "spec": {"containers": [{"name": "c", "image": "kubernetes-amd/pause"}]}}


def test_eviction_decrements_the_budget_and_races_cannot_overspend(run):
    """Three ready pods, minAvailable 2 -> one disruption allowed: of two concurrent evictions
    exactly one succeeds (the other gets 429), and the budget records the evicted pod in
    status.disruptedPods with disruptionsAllowed back at 0; a second matching budget makes the
    eviction a 500."""
    async def main():
        async with LocalCluster(nodes=1, gpus_per_node=1, controllers=["disruption"]) as cl:
            c = cl.client
            for i in range(3):
                await c.create("pods", _bare_pod(f"w{i}"))

            async def ready():
                ps = (await c.list("pods", "default", label_selector="app=web"))["items"]
                return len(ps) == 3 and all(any(x.get("type") == "Ready" and x.get("status") == "True"
                                                for x in (p.get("status") or {}).get("conditions") or ()) for p in ps)
            await cl.wait_for(ready, timeout=60)
            await c.create("poddisruptionbudgets", _pdb_obj("web", 2))

            async def allowed(n):
                st = (await c.get("poddisruptionbudgets", "web", "default")).get("status") or {}
                return st.get("disruptionsAllowed") == n and st.get("currentHealthy") == 3
            await cl.wait_for(lambda: allowed(1), timeout=30)
            res = await asyncio.gather(c.evict("default", "w0", grace_period=0), c.evict("default", "w1", grace_period=0),
                                       return_exceptions=True)
            errs = [r for r in res if isinstance(r, Exception)]
            assert len(errs) == 1 and isinstance(errs[0], APIStatusError) and errs[0].code == 429, res
            st = (await c.get("poddisruptionbudgets", "web", "default"))["status"]
            evicted = "w0" if not isinstance(res[0], Exception) else "w1"
            assert st["disruptionsAllowed"] == 0 and evicted in (st.get("disruptedPods") or {evicted: 1}), st

            async def settled():          # the pod is gone, so the controller drops its disruptedPods entry
                st = (await c.get("poddisruptionbudgets", "web", "default")).get("status") or {}
                return (st.get("currentHealthy"), st.get("disruptionsAllowed"), st.get("disruptedPods")) == (2, 0, None)
            await cl.wait_for(settled, timeout=30)
            await c.create("poddisruptionbudgets", _pdb_obj("web2", 1))
            with pytest.raises(APIStatusError) as ei:
                await c.evict("default", "w2")
            assert ei.value.code == 500
    run(main(), timeout=120)


def test_eviction_records_the_pod_and_refuses_stale_or_spent_budgets(run):
    """Without the disruption controller: a budget whose status lags its generation is a 429;
    an allowed eviction writes disruptionsAllowed - 1 and disruptedPods[pod] before deleting."""
    async def main():
        async with LocalCluster(nodes=1, gpus_per_node=1) as cl:
            c = cl.client
            for i in range(2):
                await c.create("pods", _bare_pod(f"w{i}"))
            b = await c.create("poddisruptionbudgets", _pdb_obj("web", 0))
            with pytest.raises(APIStatusError) as ei:        # no status yet: observedGeneration 0 < 1
                await c.evict("default", "w0")
            assert ei.value.code == 429
            st = {"observedGeneration": b["metadata"].get("generation", 1), "disruptionsAllowed": 1,
                  "currentHealthy": 2, "desiredHealthy": 0, "expectedPods": 2}
            await c.patch("poddisruptionbudgets", "web", {"status": st}, "default", "merge", "status")
            await c.evict("default", "w0")
            st = (await c.get("poddisruptionbudgets", "web", "default"))["status"]
            assert st["disruptionsAllowed"] == 0 and list(st["disruptedPods"]) == ["w0"]
            with pytest.raises(APIStatusError) as ei:
                await c.evict("default", "w1")
            assert ei.value.code == 429
    run(main(), timeout=90)


def test_eviction_retries_only_the_delete_on_a_stale_worker(run):
    """Shared store: when the worker's view of the pod is stale at the delete (another worker
    changed it after the budget check), only the delete is retried — the budget is decremented
    once, not again by a re-run of the whole eviction."""
    from kubernetes_amd.apiserver import server as srv_mod
    from kubernetes_amd.apiserver.server import APIServer
    from kubernetes_amd.client.rest import Client
    from kubernetes_amd.storage.remote import StoreServer

    async def main():
        store = StoreServer()
        addr = store.start()
        s = APIServer(store=addr)
        port = await s.start()
        c = Client(f"http://127.0.0.1:{port}")
        try:
            for i in range(2):
                await c.create("pods", _bare_pod(f"w{i}"))
            b = await c.create("poddisruptionbudgets", _pdb_obj("web", 0))
            st = {"observedGeneration": b["metadata"].get("generation", 1), "disruptionsAllowed": 2,
                  "currentHealthy": 2, "desiredHealthy": 0, "expectedPods": 2}
            await c.patch("poddisruptionbudgets", "web", {"status": st}, "default", "merge", "status")
            orig = s.delete
            calls = []

            async def stale_once(ri, ns, name, opts, user=None):
                calls.append(name)
                if len(calls) == 1 and ri.plural == "pods":
                    raise srv_mod._Stale(0)        # the pod changed under this worker's cache
                return await orig(ri, ns, name, opts, user)
            s.delete = stale_once
            await c.evict("default", "w0")
            st = (await c.get("poddisruptionbudgets", "web", "default"))["status"]
            assert st["disruptionsAllowed"] == 1, st          # spent once, not twice
            assert list(st["disruptedPods"]) == ["w0"]
            assert calls == ["w0", "w0"]
            names = [p["metadata"]["name"] for p in (await c.list("pods", "default"))["items"]]
            assert "w0" not in names or any(p["metadata"].get("deletionTimestamp")
                                            for p in (await c.list("pods", "default"))["items"])
        finally:
            await c.close()
            await s.stop()
            store.stop()
    run(main(), timeout=60)
