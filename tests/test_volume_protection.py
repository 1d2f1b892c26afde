"""PVC / PV protection controllers (`pkg/controller/volume/pvcprotection/
pvc_protection_controller_test.go`, `pvprotection/pv_protection_controller_test.go`): the
finalizer stays while the object is in use and is removed once it is not."""
import asyncio

from kubernetes_amd.client.fake import FakeClient
from kubernetes_amd.client.informer import InformerFactory
from kubernetes_amd.controllers.volume import (PV_PROTECTION, PVC_PROTECTION, PVCProtectionController,
                                               PVProtectionController)

DEL = "2000-01-01T00:00:00Z"


def pvc(deleting=True, fins=(PVC_PROTECTION,)):
    o = {"apiVersion": "v1", "kind": "PersistentVolumeClaim",
         "metadata": {"name": "claim", "namespace": "default", "finalizers": list(fins)}}
    if deleting:
        o["metadata"]["deletionTimestamp"] = DEL
    return o


def pod(node="node-1", phase="Running", deleting=False, statuses=None):
    p = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "p", "namespace": "default"},
         "spec": {"volumes": [{"name": "v", "persistentVolumeClaim": {"claimName": "claim"}}]},
         "status": {"phase": phase}}
    if node:
        p["spec"]["nodeName"] = node
    if deleting:
        p["metadata"]["deletionTimestamp"] = DEL
    if statuses is not None:
        p["status"]["containerStatuses"] = statuses
    return p


def run_pvc(*objs):
    async def main():
        c = FakeClient(*objs)
        f = InformerFactory(c)
        ctl = PVCProtectionController(c, f)
        ctl.setup()
        f.start()
        await f.wait_for_cache_sync()
        await ctl.sync("default/claim")
        return c.objects["persistentvolumeclaims"][("default", "claim")]["metadata"].get("finalizers") or []
    return asyncio.run(main())


def test_pvc_finalizer_kept_while_a_scheduled_running_pod_uses_it():
    assert run_pvc(pvc(), pod()) == [PVC_PROTECTION]


def test_pvc_finalizer_removed_when_unused_unscheduled_or_terminated():
    assert run_pvc(pvc()) == []
    assert run_pvc(pvc(), pod(node=None)) == []                          # unscheduled: does not block
    assert run_pvc(pvc(), pod(phase="Succeeded")) == []
    running = [{"name": "c", "state": {"running": {}}}]
    stopped = [{"name": "c", "state": {"terminated": {"exitCode": 0}}}]
    assert run_pvc(pvc(), pod(deleting=True, statuses=running)) == [PVC_PROTECTION]
    assert run_pvc(pvc(), pod(deleting=True, statuses=stopped)) == []


def test_live_pvc_gets_the_finalizer():
    assert run_pvc(pvc(deleting=False, fins=())) == [PVC_PROTECTION]


def run_pv(phase):
    async def main():
        pv = {"apiVersion": "v1", "kind": "PersistentVolume",
              "metadata": {"name": "vol", "finalizers": [PV_PROTECTION, "other"], "deletionTimestamp": DEL},
              "spec": {}, "status": {"phase": phase}}
        c = FakeClient(pv)
        f = InformerFactory(c)
        ctl = PVProtectionController(c, f)
        ctl.setup()
        f.start()
        await f.wait_for_cache_sync()
        assert len(ctl.queue) == 1
        await ctl.sync("vol")
        return c.objects["persistentvolumes"][(None, "vol")]["metadata"].get("finalizers")
    return asyncio.run(main())


def test_pv_finalizer_kept_while_bound_and_removed_after():
    assert run_pv("Bound") == [PV_PROTECTION, "other"]
    assert run_pv("Released") == ["other"]
