"""CSI end to end: host-path CSI driver (Identity/Controller/Node over a unix socket, v0.1
wire format), attach/detach controller → VolumeAttachment → external attacher
(ControllerPublishVolume) → kubelet WaitForAttach + NodePublishVolume → pod sees the data →
pod deletion unpublishes and detaches. Reference: pkg/volume/csi/*_test.go,
pkg/controller/volume/attachdetach."""
import os

from kubernetes_amd.cluster import LocalCluster
from kubernetes_amd.csi import api as CSI
from kubernetes_amd.csi.driver import CSIClient, HostPathDriver


def test_csi_wire_and_driver(run, tmp_path):
    async def main():
        drv = await HostPathDriver("hostpath.csi.amd.com", str(tmp_path / "data"), "node-0").start(str(tmp_path / "csi.sock"))
        c = CSIClient(str(tmp_path / "csi.sock"))
        try:
            await c.assert_supported_version()
            info = await c.controller_publish("vol-1", "node-0")
            assert info["devicePath"].endswith("vol-1")
            try:
                await c.controller_publish("vol-1", "node-1")         # RWO: second node refused
                raise AssertionError("expected FAILED_PRECONDITION")
            except Exception as e:
                assert "already published" in str(e)
            tgt = str(tmp_path / "pod" / "mount")
            await c.node_publish("vol-1", tgt, publish_info=info)
            with open(os.path.join(tgt, "f"), "w") as f:
                f.write("hi")
            assert os.path.exists(os.path.join(info["devicePath"], "f"))
            await c.node_unpublish("vol-1", tgt)
            assert not os.path.exists(tgt)
            await c.controller_unpublish("vol-1", "node-0")
            assert "vol-1" not in drv.attached
        finally:
            await c.close()
            await drv.stop()
    run(main())


def test_csi_attach_publish_end_to_end(run):
    import shutil
    import tempfile
    from pathlib import Path
    tmp_path = Path(tempfile.mkdtemp(prefix="csi", dir="/tmp"))       # unix socket paths are <108 chars

    async def main():
        driver = "hostpath.csi.amd.com"
        cl = LocalCluster(nodes=1, gpus_per_node=0, runtime="process", workdir=str(tmp_path / "c"),
                          controllers=["attachdetach", "persistentvolume-binder", "csi-attacher"],
                          controller_options={"csi-attacher": {"driver": driver,
                                                               "endpoint": str(tmp_path / "ctrl.sock")}})
        # one driver process serves the controller socket, the node plugin serves the kubelet's
        node_sock = CSI.socket_path(os.path.join(str(tmp_path / "c"), "node-0", "plugins"), driver)
        drv = await HostPathDriver(driver, str(tmp_path / "data"), "node-0").start(str(tmp_path / "ctrl.sock"))
        drv2 = await HostPathDriver(driver, str(tmp_path / "data"), "node-0").start(node_sock)
        await cl.start()
        c = cl.client
        try:
            # 1.9's CSIPersistentVolumeSource has no volumeAttributes: they ride on an annotation
            await c.create("persistentvolumes", {"metadata": {"name": "csi-pv", "annotations": {
                "csi.volume.kubernetes.io/volume-attributes": '{"tier": "nvme"}'}}, "spec": {
                "capacity": {"storage": "10Gi"}, "accessModes": ["ReadWriteOnce"], "storageClassName": "",
                "csi": {"driver": driver, "volumeHandle": "dataset-7"}}})
            await c.create("persistentvolumeclaims", {"metadata": {"name": "data"}, "spec": {
                "accessModes": ["ReadWriteOnce"], "storageClassName": "", "resources": {"requests": {"storage": "1Gi"}}}},
                "default")
            await c.create("pods", {"metadata": {"name": "reader"}, "spec": {
                "containers": [{"name": "c", "image": "busybox", "command": ["sh", "-c", "sleep 30"],
                                "volumeMounts": [{"name": "d", "mountPath": "/data"}]}],
                "volumes": [{"name": "d", "persistentVolumeClaim": {"claimName": "data"}}]}}, "default")
            va_name = CSI.attachment_name("csi-pv", driver, "node-0")

            async def attached():
                try:
                    va = await c.get("volumeattachments", va_name)
                except Exception:
                    return None
                return va if (va.get("status") or {}).get("attached") else None
            va = await cl.wait_for(attached, 20)
            assert va["spec"]["nodeName"] == "node-0" and drv.attached == {"dataset-7": "node-0"}

            async def published():
                return drv2.published.get("dataset-7") or None
            targets = await cl.wait_for(published, 20)
            assert any("kubernetes.io~csi/csi-pv/mount" in t for t in targets)

            async def node_reports():
                n = await c.get("nodes", "node-0")
                return [v["name"] for v in (n.get("status") or {}).get("volumesAttached") or ()]
            names = await cl.wait_for(node_reports, 10)
            assert names == [f"kubernetes.io/csi/{driver}^dataset-7"]
            await c.delete("pods", "reader", "default", grace_period=0)

            async def detached():
                try:
                    await c.get("volumeattachments", va_name)
                    return False
                except Exception:
                    return not drv.attached and not drv2.published.get("dataset-7")
            try:
                await cl.wait_for(detached, 20)
            except TimeoutError:
                vas = (await c.list("volumeattachments"))["items"]
                pods = (await c.list("pods", "default"))["items"]
                raise AssertionError(f"vas={[v['metadata']['name'] for v in vas]} attached={drv.attached} "
                                     f"published={drv2.published} pods={[p['metadata'] for p in pods]}")
        finally:
            await cl.stop()
            await drv.stop()
            await drv2.stop()
    try:
        run(main(), timeout=90)
    finally:
        shutil.rmtree(tmp_path, ignore_errors=True)
