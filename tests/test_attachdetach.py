"""Attach/detach controller reconciler (`pkg/controller/volume/attachdetach/reconciler/
reconciler_test.go` behaviours) over the fake client: attach for scheduled pods on nodes that
hand attach/detach to the controller, never detach a volume the node still reports in
`volumesInUse` until maxWaitForUnmountDuration, Multi-Attach errors for single-node volumes,
and `node.status.volumesAttached` kept equal to the attached set."""
import asyncio

from kubernetes_amd.client.fake import FakeClient
from kubernetes_amd.client.informer import InformerFactory
from kubernetes_amd.controllers.attachdetach import (CONTROLLER_MANAGED_ATTACH, AttachDetachController,
                                                     unique_volume_name)
from kubernetes_amd.csi import api as CSI

DRIVER = "csi.example.com"


def node(name, managed=True, in_use=()):
    n = {"apiVersion": "v1", "kind": "Node", "metadata": {"name": name}, "status": {}}
    if managed:
        n["metadata"]["annotations"] = {CONTROLLER_MANAGED_ATTACH: "true"}
    if in_use:
        n["status"]["volumesInUse"] = list(in_use)
    return n


def pv(name, modes=("ReadWriteOnce",)):
    return {"apiVersion": "v1", "kind": "PersistentVolume", "metadata": {"name": name},
            "spec": {"accessModes": list(modes), "capacity": {"storage": "1Gi"},
                     "csi": {"driver": DRIVER, "volumeHandle": f"h-{name}"}}}


def pvc(name, volume):
    return {"apiVersion": "v1", "kind": "PersistentVolumeClaim", "metadata": {"name": name, "namespace": "default"},
            "spec": {"volumeName": volume}, "status": {"phase": "Bound"}}


def pod(name, node_name, claim, phase="Running"):
    return {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "namespace": "default", "uid": f"{name}-uid"},
            "spec": {"nodeName": node_name, "volumes": [{"name": "v", "persistentVolumeClaim": {"claimName": claim}}]},
            "status": {"phase": phase}}


def va(pv_name, node_name, attached=True):
    name = CSI.attachment_name(pv_name, DRIVER, node_name)
    return {"apiVersion": "storage.k8s.io/v1beta1", "kind": "VolumeAttachment", "metadata": {"name": name},
            "spec": {"attacher": DRIVER, "nodeName": node_name, "source": {"persistentVolumeName": pv_name}},
            "status": {"attached": attached}}


def reconcile(*objs, max_wait=360.0, rounds=1, between=None):
    async def main():
        c = FakeClient(*objs)
        f = InformerFactory(c)
        ctl = AttachDetachController(c, f)
        ctl.max_wait_for_unmount = max_wait
        ctl.setup()
        events = []
        ctl.recorder.event = lambda obj, typ, reason, msg: events.append((obj["metadata"]["name"], reason))
        f.start()
        await f.wait_for_cache_sync()
        for i in range(rounds):
            await ctl.sync("reconcile")
            if between:
                await between(c, i)
                await asyncio.sleep(0.05)
        return c, events
    return asyncio.run(main())


def _vas(c):
    return sorted(o["metadata"]["name"] for o in c.objects.get("volumeattachments", {}).values())


def test_attach_for_pods_on_managed_nodes_only():
    c, _ = reconcile(node("n1"), node("n2", managed=False), pv("a"), pv("b"), pvc("ca", "a"), pvc("cb", "b"),
                     pod("p1", "n1", "ca"), pod("p2", "n2", "cb"))
    assert _vas(c) == [CSI.attachment_name("a", DRIVER, "n1")]


def test_terminated_pods_do_not_keep_volumes_attached():
    c, _ = reconcile(node("n1"), pv("a"), pvc("ca", "a"), pod("p1", "n1", "ca", phase="Succeeded"), va("a", "n1"))
    assert _vas(c) == []


def test_no_detach_while_the_node_reports_the_volume_in_use():
    in_use = unique_volume_name(DRIVER, "h-a")
    c, _ = reconcile(node("n1", in_use=[in_use]), pv("a"), va("a", "n1"))
    assert _vas(c) == [CSI.attachment_name("a", DRIVER, "n1")]          # still mounted: kept

    async def unmounted(c, i):
        if i == 0:
            await c.patch("nodes", "n1", {"status": {"volumesInUse": None}}, None, "merge", "status")
    c, _ = reconcile(node("n1", in_use=[in_use]), pv("a"), va("a", "n1"), rounds=2, between=unmounted)
    assert _vas(c) == []


def test_force_detach_after_max_wait_for_unmount():
    in_use = unique_volume_name(DRIVER, "h-a")

    async def wait(c, i):
        await asyncio.sleep(0.1)
    c, _ = reconcile(node("n1", in_use=[in_use]), pv("a"), va("a", "n1"), max_wait=0.05, rounds=2, between=wait)
    assert _vas(c) == []


def test_multi_attach_error_for_single_node_volumes():
    c, events = reconcile(node("n1"), node("n2"), pv("a"), pvc("ca", "a"), pod("p1", "n1", "ca"),
                          pod("p2", "n2", "ca"), va("a", "n1"))
    assert _vas(c) == [CSI.attachment_name("a", DRIVER, "n1")]
    assert events == [("p2", "FailedAttachVolume")]
    c, events = reconcile(node("n1"), node("n2"), pv("rwx", ("ReadWriteMany",)), pvc("cx", "rwx"),
                          pod("p1", "n1", "cx"), pod("p2", "n2", "cx"), va("rwx", "n1"))
    assert len(_vas(c)) == 2 and not events


def test_node_status_volumes_attached_tracks_the_actual_state():
    c, _ = reconcile(node("n1"), pv("a"), pvc("ca", "a"), pod("p1", "n1", "ca"), va("a", "n1"))
    n1 = c.objects["nodes"][(None, "n1")]
    assert [v["name"] for v in n1["status"]["volumesAttached"]] == [unique_volume_name(DRIVER, "h-a")]
    stale = node("n1")
    stale["status"]["volumesAttached"] = [{"name": unique_volume_name(DRIVER, "h-gone"), "devicePath": ""}]
    c, _ = reconcile(stale)
    assert not c.objects["nodes"][(None, "n1")]["status"].get("volumesAttached")


def test_kubelet_reports_volumes_in_use(tmp_path):
    """The kubelet side of the handshake: a CSI volume is reported in use before it is mounted
    and dropped when the pod's volumes are torn down; the node advertises that the controller
    attaches its volumes."""
    from kubernetes_amd.kubelet.volumes import VolumeManager
    vm = VolumeManager(None, str(tmp_path / "pods"), str(tmp_path / "plugins"), "n1")
    changes = []
    vm.on_in_use_change = lambda: changes.append(1)
    p = pod("p1", "n1", "ca")
    vm._mark_in_use(p, unique_volume_name(DRIVER, "h-a"))
    vm._mark_in_use(p, unique_volume_name(DRIVER, "h-a"))
    assert vm.volumes_in_use() == [unique_volume_name(DRIVER, "h-a")] and len(changes) == 1
    asyncio.run(vm.unpublish(p))
    assert vm.volumes_in_use() == [] and len(changes) == 2
    from kubernetes_amd.kubelet.kubelet import CONTROLLER_MANAGED_ATTACH as KUBELET_ANN
    assert KUBELET_ANN == CONTROLLER_MANAGED_ATTACH
