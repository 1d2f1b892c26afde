"""Pod GC: `pkg/controller/podgc/gc_controller_test.go` — TestGCTerminated (the oldest
terminated pods beyond the threshold, none when the threshold is 0), TestGCOrphaned (pods on
nodes that no longer exist) and TestGCUnscheduledTerminating (terminating pods that were never
scheduled)."""
import asyncio

import pytest

from kubernetes_amd.client.fake import FakeClient
from kubernetes_amd.client.informer import InformerFactory
from kubernetes_amd.controllers.lifecycle import PodGCController


def pod(name, phase="Running", node="node", created="2017-01-01T00:00:00Z", deleting=False):
    p = {"apiVersion": "v1", "kind": "Pod",
         "metadata": {"name": name, "namespace": "default", "creationTimestamp": created},
         "spec": {"nodeName": node} if node else {}, "status": {"phase": phase}}
    if deleting:
        p["metadata"]["deletionTimestamp"] = "2017-01-01T00:00:00Z"
    return p


def node(name):
    return {"apiVersion": "v1", "kind": "Node", "metadata": {"name": name}}


def run_gc(objs, threshold):
    async def main():
        c = FakeClient(*objs)
        f = InformerFactory(c)
        gc = PodGCController(c, f, terminated_pod_gc_threshold=threshold)
        gc.setup()
        f.start()
        await f.wait_for_cache_sync()
        await gc.sync("gc")
        return sorted(a.name for a in c.actions if a.verb == "delete" and a.resource == "pods")
    return asyncio.run(main())


@pytest.mark.parametrize("phases,threshold,deleted", [
    (["Failed", "Failed"], 1, ["a"]),
    (["Failed", "Succeeded"], 0, []),
    (["Failed"], 1, []),
    (["Failed", "Succeeded", "Running"], 1, ["a"]),
    (["Failed", "Running", "Succeeded"], 1, ["a"]),
    (["Failed", "Failed", "Succeeded", "Running"], 1, ["a", "b"])])
def test_gc_terminated(phases, threshold, deleted):
    objs = [node("node")] + [pod(chr(ord("a") + i), ph, created=f"2017-01-01T00:00:0{i}Z") for i, ph in enumerate(phases)]
    assert run_gc(objs, threshold) == deleted


def test_gc_orphaned():
    objs = [node("node"), pod("a", node="node"), pod("b", node="gone")]
    assert run_gc(objs, 10) == ["b"]


def test_gc_unscheduled_terminating():
    objs = [node("node"), pod("a", node="", deleting=True), pod("b", node="node", deleting=True), pod("c", node="")]
    assert run_gc(objs, 10) == ["a"]
