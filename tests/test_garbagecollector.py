"""Garbage collector: tables ported from `pkg/controller/garbagecollector/garbagecollector_test.go`
(TestProcessEvent + verifyGraphInvariants, TestAttemptToDeleteItem, TestAbsentUIDCache,
TestDeleteOwnerRefPatch, TestUnblockOwnerReference, TestGetDeletableResources) plus live-cluster
cases for what the table tests do not reach: owners of every kind (custom resources, PVCs,
service accounts) are confirmed with a live GET before a dependent is collected; foreground
deletion waits for blocking dependents; orphaning strips the references.
"""
import asyncio
import copy
import json

import pytest

from kubernetes_amd.client.fake import FakeClient
from kubernetes_amd.client.informer import InformerFactory
from kubernetes_amd.cluster import LocalCluster
from kubernetes_amd.controllers.garbagecollector import (GarbageCollector, Node, UIDCache, delete_owner_ref_patch,
                                                         deletable_resources)
from kubernetes_amd.utils.patch import apply_patch

SMP = "application/strategic-merge-patch+json"


def _gc(client=None):
    client = client or FakeClient()
    gc = GarbageCollector(client, InformerFactory(client))
    gc.setup()
    return gc


def _pod(uid, owners, name=None):
    return {"apiVersion": "v1", "kind": "Pod",
            "metadata": {"name": name or f"p{uid}", "namespace": "ns1", "uid": uid,
                         "ownerReferences": [{"uid": o, "apiVersion": "v1", "kind": "Pod", "name": f"p{o}"}
                                             for o in owners]}}


def _invariants(graph):
    """verifyGraphInvariants: dependents <-> owners agree in both directions."""
    for uid, n in graph.items():
        for du in n.dependents:
            dep = graph[du]
            assert any(r.get("uid") == uid for r in dep.owners), f"{n} lists {dep} but is not its owner"
        for ref in n.owners:
            on = graph.get(ref["uid"])
            if on is not None:
                assert n.uid in on.dependents, f"{n} has owner {on} that does not list it"


SCENARIOS = {
    "test1": [("add", "1", []), ("add", "2", ["1"]), ("add", "3", ["1", "2"])],
    "test2": [("add", "1", []), ("add", "2", ["1"]), ("add", "3", ["1", "2"]), ("add", "4", ["2"]),
              ("delete", "2", ["doesn't matter"])],
    "test3": [("add", "1", []), ("add", "2", ["1"]), ("add", "3", ["1", "2"]), ("add", "4", ["3"]),
              ("update", "2", ["4"])],
    "reverse test2": [("add", "4", ["2"]), ("add", "3", ["1", "2"]), ("add", "2", ["1"]), ("add", "1", []),
                      ("delete", "2", ["doesn't matter"])],
}


@pytest.mark.parametrize("name", list(SCENARIOS))
def test_process_event_graph_invariants(name, run):
    async def main():
        gc = _gc()
        for etype, uid, owners in SCENARIOS[name]:
            gc._on_event(etype, "v1", "Pod", _pod(uid, owners), None)
            _invariants(gc.graph)
        return gc
    gc = run(main())
    if name == "test2":
        assert "2" not in gc.graph and gc.graph["4"].owners[0]["uid"] == "2"
        # dependents of the deleted node were queued for attemptToDelete
        assert "d|4" in gc.queue._queue and "d|3" in gc.queue._queue
    if name == "reverse test2":
        # "1" started virtual (referenced before observed) and became observed on its add event
        assert not gc.graph["1"].virtual


def test_virtual_owner_is_queued_for_verification(run):
    async def main():
        gc = _gc()
        gc._on_event("add", "v1", "Pod", _pod("2", ["1"]), None)
        n = gc.graph["1"]
        assert n.virtual and n.namespace == "ns1" and n.kind == "Pod" and n.name == "p1"
        assert "d|1" in gc.queue._queue
    run(main())


def test_attempt_to_delete_item(run):
    """TestAttemptToDeleteItem: owner GET 404 -> the dependent is deleted (background, UID precondition)."""
    async def main():
        pod = _pod("456", [])
        pod["metadata"]["name"] = "ToBeDeletedPod"
        pod["metadata"]["ownerReferences"] = [{"kind": "ReplicationController", "name": "owner1", "uid": "123",
                                               "apiVersion": "v1"}]
        c = FakeClient(pod)
        gc = _gc(c)
        item = Node("456", "v1", "Pod", "ns1", "ToBeDeletedPod")   # owners left empty on purpose
        deletes = []
        orig = c.delete

        async def delete(resource, name, namespace=None, grace_period=None, propagation=None, uid=None, decode=True):
            deletes.append((propagation, uid))
            return await orig(resource, name, namespace, grace_period, propagation, uid, decode)
        c.delete = delete
        await gc.attempt_to_delete_item(item)
        acts = {f"{a.verb}={a.resource}/{a.namespace}/{a.name}" for a in c.actions}
        assert acts == {"get=replicationcontrollers/ns1/owner1", "get=pods/ns1/ToBeDeletedPod",
                        "delete=pods/ns1/ToBeDeletedPod"}
        assert ("Background", "456") in deletes
    run(main())


def test_attempt_to_delete_keeps_dependent_of_live_owner(run):
    async def main():
        rc = {"apiVersion": "v1", "kind": "ReplicationController",
              "metadata": {"name": "owner1", "namespace": "ns1", "uid": "123"}}
        pod = _pod("456", [])
        pod["metadata"]["ownerReferences"] = [{"kind": "ReplicationController", "name": "owner1", "uid": "123",
                                               "apiVersion": "v1"}]
        c = FakeClient(rc, pod)
        gc = _gc(c)
        await gc.attempt_to_delete_item(Node("456", "v1", "Pod", "ns1", "p456"))
        assert not [a for a in c.actions if a.verb in ("delete", "patch")]
        # same name, different UID: the owner was recreated -> dangling -> collected
        rc2 = copy.deepcopy(rc)
        c.objects["replicationcontrollers"][("ns1", "owner1")]["metadata"]["uid"] = "999"
        await gc.attempt_to_delete_item(Node("456", "v1", "Pod", "ns1", "p456"))
        assert [a for a in c.actions if a.verb == "delete"], rc2
    run(main())


def test_solid_and_dangling_owners_patch_away_the_dangling_reference(run):
    async def main():
        rc = {"apiVersion": "v1", "kind": "ReplicationController",
              "metadata": {"name": "live", "namespace": "ns1", "uid": "1"}}
        pod = _pod("9", [])
        pod["metadata"]["ownerReferences"] = [
            {"kind": "ReplicationController", "name": "live", "uid": "1", "apiVersion": "v1"},
            {"kind": "ReplicationController", "name": "gone", "uid": "2", "apiVersion": "v1"}]
        c = FakeClient(rc, pod)
        gc = _gc(c)
        await gc.attempt_to_delete_item(Node("9", "v1", "Pod", "ns1", "p9"))
        assert not [a for a in c.actions if a.verb == "delete"]
        patched = await c.get("pods", "p9", "ns1")
        assert [r["uid"] for r in patched["metadata"]["ownerReferences"]] == ["1"]
    run(main())


def test_absent_uid_cache(run):
    """TestAbsentUIDCache: a cached-absent owner is not fetched again; LRU eviction at size 2."""
    async def main():
        def rcpod(name, rc, uid):
            p = _pod(name, [], name=name)
            p["metadata"]["ownerReferences"] = [{"kind": "ReplicationController", "name": rc, "uid": uid,
                                                 "apiVersion": "v1"}]
            return p
        pods = [rcpod("rc1Pod1", "rc1", "1"), rcpod("rc1Pod2", "rc1", "1"), rcpod("rc2Pod1", "rc2", "2"),
                rcpod("rc3Pod1", "rc3", "3")]
        c = FakeClient(*pods)
        c.prepend_reactor("delete", "pods", lambda a: (True, {"kind": "Status"}))   # keep the pods
        gc = _gc(c)
        gc.absent = UIDCache(2)
        for name in ("rc1Pod1", "rc2Pod1", "rc1Pod2", "rc3Pod1"):
            await gc.attempt_to_delete_item(Node(name, "v1", "Pod", "ns1", name))
        assert gc.absent.has("1") and not gc.absent.has("2") and gc.absent.has("3")
        gets = [a for a in c.actions if a.verb == "get" and a.resource == "replicationcontrollers" and a.name == "rc1"]
        assert len(gets) == 1
    run(main())


def test_delete_owner_ref_patch():
    """TestDeleteOwnerRefPatch: the strategic-merge patch drops exactly the named owners."""
    original = {"metadata": {"uid": "100", "ownerReferences": [{"uid": "1"}, {"uid": "2"}, {"uid": "3"}]}}
    patch = delete_owner_ref_patch("100", "2", "3")
    got = apply_patch(SMP, copy.deepcopy(original), json.loads(json.dumps(patch)))
    assert got == {"metadata": {"uid": "100", "ownerReferences": [{"uid": "1"}]}}


def test_unblock_owner_reference():
    """TestUnblockOwnerReference."""
    original = {"metadata": {"uid": "100", "ownerReferences": [
        {"uid": "1", "blockOwnerDeletion": True}, {"uid": "2", "blockOwnerDeletion": False}, {"uid": "3"}]}}
    n = Node("100", "v1", "Pod", "ns", "p", owners=original["metadata"]["ownerReferences"])
    got = apply_patch(SMP, copy.deepcopy(original), n.unblock_patch())
    assert got["metadata"]["ownerReferences"] == [
        {"uid": "1", "blockOwnerDeletion": False}, {"uid": "2", "blockOwnerDeletion": False}, {"uid": "3"}]


def test_get_deletable_resources():
    """TestGetDeletableResources (+ preferred-version choice and alias de-duplication)."""
    lists = [
        {"groupVersion": "apps/v1", "resources": [
            {"name": "pods", "namespaced": True, "kind": "Pod", "verbs": ["delete", "list", "watch"]},
            {"name": "services", "namespaced": True, "kind": "Service"}]},
        {"groupVersion": "foo//whatever", "resources": [
            {"name": "bars", "namespaced": True, "kind": "Bar", "verbs": ["delete", "list", "watch"]}]},
        {"groupVersion": "acme/v1", "resources": [
            {"name": "widgets", "namespaced": True, "kind": "Widget", "verbs": ["delete"]}]},
    ]
    assert [(r.group, r.version, r.plural) for r in deletable_resources(lists)] == [("apps", "v1", "pods")]
    assert deletable_resources([]) == []
    verbs = ["create", "delete", "list", "watch", "get"]
    lists = [
        {"groupVersion": "v1", "resources": [
            {"name": "events", "kind": "Event", "namespaced": True, "verbs": verbs},
            {"name": "pods", "kind": "Pod", "namespaced": True, "verbs": verbs},
            {"name": "pods/status", "kind": "Pod", "namespaced": True, "verbs": verbs}]},
        {"groupVersion": "batch/v1", "resources": [{"name": "jobs", "kind": "Job", "namespaced": True, "verbs": verbs}]},
        {"groupVersion": "batch/v1beta1", "resources": [
            {"name": "cronjobs", "kind": "CronJob", "namespaced": True, "verbs": verbs}]},
        {"groupVersion": "batch/v2alpha1", "resources": [
            {"name": "cronjobs", "kind": "CronJob", "namespaced": True, "verbs": verbs}]},
        {"groupVersion": "extensions/v1beta1", "resources": [
            {"name": "deployments", "kind": "Deployment", "namespaced": True, "verbs": verbs},
            {"name": "ingresses", "kind": "Ingress", "namespaced": True, "verbs": verbs}]},
        {"groupVersion": "apiextensions.k8s.io/v1beta1", "resources": [
            {"name": "customresourcedefinitions", "kind": "CustomResourceDefinition", "namespaced": False,
             "verbs": verbs}]},
    ]
    got = [(r.group, r.version, r.plural) for r in deletable_resources(lists)]
    assert got == [("", "v1", "pods"), ("batch", "v1", "jobs"), ("batch", "v1beta1", "cronjobs"),
                   ("extensions", "v1beta1", "ingresses")]


# -- live cluster -----------------------------------------------------------------------------

WIDGET_CRD = {"apiVersion": "apiextensions.k8s.io/v1beta1", "kind": "CustomResourceDefinition",
              "metadata": {"name": "widgets.example.com"},
              "spec": {"group": "example.com", "version": "v1", "scope": "Namespaced",
                       "names": {"plural": "widgets", "singular": "widget", "kind": "Widget"}}}


def _cm(name, owner, api_version, kind, block=None):
    ref = {"apiVersion": api_version, "kind": kind, "name": owner["metadata"]["name"], "uid": owner["metadata"]["uid"]}
    if block is not None:
        ref["blockOwnerDeletion"] = block
    return {"apiVersion": "v1", "kind": "ConfigMap",
            "metadata": {"name": name, "namespace": "default", "ownerReferences": [ref]}, "data": {"k": "v"}}


async def _exists(c, res, name, ns="default"):
    try:
        await c.get(res, name, ns)
        return True
    except Exception:
        return False


def test_live_owners_of_any_kind_keep_their_dependents(run):
    """The round-4 data-loss probe: a ConfigMap owned by a live custom resource (and by a PVC, a
    ServiceAccount) must survive; once the owner is deleted, the dependent is collected."""
    async def main():
        async with LocalCluster(nodes=1, gpus_per_node=1, controllers=["garbagecollector"],
                                controller_options={"garbagecollector": {"discovery_period": 1.0}}) as cl:
            c = cl.client
            await c.create("customresourcedefinitions", copy.deepcopy(WIDGET_CRD))
            st, body = await c.raw("POST", "/apis/example.com/v1/namespaces/default/widgets", json.dumps(
                {"apiVersion": "example.com/v1", "kind": "Widget", "metadata": {"name": "w1"}}).encode())
            assert st == 201, body
            widget = json.loads(body)
            sa = await c.create("serviceaccounts", {"metadata": {"name": "owner-sa", "namespace": "default"}})
            pvc = await c.create("persistentvolumeclaims", {"metadata": {"name": "owner-pvc", "namespace": "default"},
                                 "spec": {"accessModes": ["ReadWriteOnce"],
                                          "resources": {"requests": {"storage": "1Gi"}}}})
            await c.create("configmaps", _cm("of-widget", widget, "example.com/v1", "Widget"))
            await c.create("configmaps", _cm("of-sa", sa, "v1", "ServiceAccount"))
            await c.create("configmaps", _cm("of-pvc", pvc, "v1", "PersistentVolumeClaim"))
            gone_owner = {"metadata": {"name": "never", "uid": "00000000-dead-beef-0000-000000000000"}}
            await c.create("configmaps", _cm("of-nothing", gone_owner, "v1", "Secret"))
            two = _cm("of-sa-and-nothing", sa, "v1", "ServiceAccount")
            two["metadata"]["ownerReferences"].append(_cm("x", gone_owner, "v1", "Secret")["metadata"]["ownerReferences"][0])
            await c.create("configmaps", two)

            async def dangling_ref_dropped():
                cm = await c.get("configmaps", "of-sa-and-nothing", "default")
                return [r["name"] for r in cm["metadata"]["ownerReferences"]] == ["owner-sa"]
            await cl.wait_for(dangling_ref_dropped, timeout=20)
            # the dangling one goes; the others stay (well past the 4 s the old collector needed)
            await cl.wait_for(lambda: _gone(c, "of-nothing"), timeout=20)
            await asyncio.sleep(3.0)
            for name in ("of-widget", "of-sa", "of-pvc"):
                assert await _exists(c, "configmaps", name), name
            gc = cl.cm.get("garbagecollector")
            assert any(ri.plural == "widgets" for ri in gc.monitors), "custom resources are monitored"
            # owners go -> dependents go
            st, _ = await c.raw("DELETE", "/apis/example.com/v1/namespaces/default/widgets/w1")
            assert st == 200
            await c.delete("serviceaccounts", "owner-sa", "default")
            await cl.wait_for(lambda: _gone(c, "of-widget"), timeout=20)
            await cl.wait_for(lambda: _gone(c, "of-sa"), timeout=20)
            await cl.wait_for(lambda: _gone(c, "of-sa-and-nothing"), timeout=20)
            assert await _exists(c, "configmaps", "of-pvc")
    run(main(), timeout=90)


async def _gone(c, name):
    return not await _exists(c, "configmaps", name)


def _rs(name, replicas=2):
    return {"apiVersion": "apps/v1", "kind": "ReplicaSet", "metadata": {"name": name, "namespace": "default"},
            "spec": {"replicas": replicas, "selector": {"matchLabels": {"app": name}},
                     "template": {"metadata": {"labels": {"app": name}},
                                  "spec": {"containers": [{"name": "c", "image": "kubernetes-amd/pause"}]}}}}


def test_foreground_and_orphan_propagation(run):
    async def main():
        async with LocalCluster(nodes=1, gpus_per_node=1, controllers=["garbagecollector", "replicaset"]) as cl:
            c = cl.client

            async def pods(app):
                return (await c.list("pods", "default", label_selector=f"app={app}"))["items"]

            async def n_pods(app, n):
                ps = [p for p in await pods(app) if not p["metadata"].get("deletionTimestamp")]
                return len(ps) == n
            # orphan: the pods stay and lose their owner reference
            await c.create("replicasets", _rs("orph"))
            await cl.wait_for(lambda: n_pods("orph", 2), timeout=30)
            await c.delete("replicasets", "orph", "default", propagation="Orphan")

            async def orphaned():
                ps = await pods("orph")
                rs_gone = not await _exists(c, "replicasets", "orph")
                return rs_gone and len(ps) == 2 and all(not p["metadata"].get("ownerReferences") for p in ps)
            await cl.wait_for(orphaned, timeout=30)
            # foreground: the owner is visible (deletionTimestamp + finalizer) until its pods are gone
            await c.create("replicasets", _rs("fg"))
            await cl.wait_for(lambda: n_pods("fg", 2), timeout=30)
            await c.delete("replicasets", "fg", "default", propagation="Foreground")
            rs = await c.get("replicasets", "fg", "default")
            assert rs["metadata"].get("deletionTimestamp") and "foregroundDeletion" in rs["metadata"]["finalizers"]

            async def fg_done():
                return not await _exists(c, "replicasets", "fg") and not await pods("fg")
            await cl.wait_for(fg_done, timeout=60)
    run(main(), timeout=150)


def test_namespace_deletion_removes_custom_resources(run):
    """The namespace controller finds what to delete through discovery, so custom resources in
    a terminating namespace are deleted too (namespaced_resources_deleter.go)."""
    async def main():
        async with LocalCluster(nodes=1, gpus_per_node=1, controllers=["namespace"]) as cl:
            c = cl.client
            await c.create("customresourcedefinitions", copy.deepcopy(WIDGET_CRD))
            await c.create("namespaces", {"metadata": {"name": "doomed"}})
            st, body = await c.raw("POST", "/apis/example.com/v1/namespaces/doomed/widgets", json.dumps(
                {"apiVersion": "example.com/v1", "kind": "Widget", "metadata": {"name": "w"}}).encode())
            assert st == 201, body
            await c.create("configmaps", {"metadata": {"name": "cm", "namespace": "doomed"}})
            await c.delete("namespaces", "doomed")

            async def gone():
                try:
                    await c.get("namespaces", "doomed")
                    return False
                except Exception:
                    return True
            await cl.wait_for(gone, timeout=30)
            st, body = await c.raw("GET", "/apis/example.com/v1/namespaces/doomed/widgets")
            assert st == 200 and json.loads(body)["items"] == []
    run(main(), timeout=60)
