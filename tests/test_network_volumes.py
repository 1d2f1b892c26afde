"""Network and block volume plugins (nfs, cephfs, glusterfs, iscsi, fc, rbd) through the kubelet
with a recording mounter — the commands and their order, formatting only blank devices, detach
on pod deletion (iSCSI logout, rbd unmap) unless another pod still uses the device, and a pod
directory that is never deleted through a mount point.

Parity: `pkg/volume/nfs/nfs_test.go`, `cephfs_test.go`, `glusterfs_test.go`, `iscsi_util_test.go`,
`rbd_test.go`, `fc_util_test.go` (FakeMounter / FakeExec doubles); `pkg/util/mount`
SafeFormatAndMount tests (format only when blkid finds nothing).
"""
import asyncio
import base64
import os

from kubernetes_amd.cluster import LocalCluster
from kubernetes_amd.kubelet.volume_plugins import FakeMounter, PluginContext, format_and_mount
from kubernetes_amd.kubelet.volumes import _rmtree_no_mounts


def _pod(name, vols, mounts=None):
    return {"metadata": {"name": name, "namespace": "default"}, "spec": {
        "volumes": vols, "containers": [{"name": "c", "image": "x", "volumeMounts": mounts or [
            {"name": v["name"], "mountPath": f"/mnt/{v['name']}"} for v in vols]}]}}


def _cmds(fm, first):
    return [c for c in fm.log if c[0] == first]


def test_filesystem_plugins_and_pv_mount_options(run):
    async def main():
        async with LocalCluster(nodes=1, gpus_per_node=0) as cl:
            c = cl.client
            fm = FakeMounter()
            cl.nodes[0].kubelet.volumes.mounter = fm
            await c.create("secrets", {"metadata": {"name": "ceph", "namespace": "default"},
                                       "data": {"key": base64.b64encode(b"AQBsecret==").decode()}})
            await c.create("endpoints", {"metadata": {"name": "gluster", "namespace": "default"},
                                         "subsets": [{"addresses": [{"ip": "10.0.0.1"}, {"ip": "10.0.0.2"}],
                                                      "ports": [{"port": 1}]}]})
            await c.create("pods", _pod("fs", [
                {"name": "data", "nfs": {"server": "fd00::5", "path": "/exports/data", "readOnly": True}},
                {"name": "ceph", "cephfs": {"monitors": ["10.1.0.1:6789", "10.1.0.2:6789"], "path": "/ml",
                                            "user": "kube", "secretRef": {"name": "ceph"}}},
                {"name": "gl", "glusterfs": {"endpoints": "gluster", "path": "vol0"}}]))
            await cl.wait_pod("fs")
            mounts = {c[-1].rsplit("/", 1)[-1]: c for c in _cmds(fm, "mount")}
            assert mounts["data"][:5] == ["mount", "-t", "nfs", "-o", "ro"] and mounts["data"][5] == "[fd00::5]:/exports/data"
            assert mounts["ceph"][1:3] == ["-t", "ceph"] and mounts["ceph"][5] == "10.1.0.1:6789,10.1.0.2:6789:/ml"
            assert mounts["ceph"][4] == "name=kube,secret=AQBsecret=="
            gl = mounts["gl"]
            assert gl[5] == "10.0.0.1:vol0" and "backup-volfile-servers=10.0.0.2" in gl[4]
            # a PV with mount options, through a claim
            await c.create("persistentvolumes", {"metadata": {"name": "nfs-pv"}, "spec": {
                "capacity": {"storage": "1Ti"}, "accessModes": ["ReadWriteMany"], "mountOptions": ["hard", "nfsvers=4.1"],
                "nfs": {"server": "nas", "path": "/ckpt"},
                "claimRef": {"namespace": "default", "name": "ckpt"}}})
            await c.create("persistentvolumeclaims", {"metadata": {"name": "ckpt", "namespace": "default"}, "spec": {
                "accessModes": ["ReadWriteMany"], "resources": {"requests": {"storage": "1Ti"}}, "volumeName": "nfs-pv"}})
            await c.patch("persistentvolumeclaims", "ckpt", {"status": {"phase": "Bound"}}, "default", "merge", "status")
            await c.create("pods", _pod("pvpod", [{"name": "ck", "persistentVolumeClaim": {"claimName": "ckpt"}}]))
            await cl.wait_pod("pvpod")
            pv = [m for m in _cmds(fm, "mount") if m[-1].endswith("kubernetes.io~nfs/nfs-pv")]
            assert pv and pv[0][1:6] == ["-t", "nfs", "-o", "hard,nfsvers=4.1", "nas:/ckpt"]
            # deletion unmounts
            await c.delete("pods", "fs", "default", grace_period=0)

            async def gone():
                return len(_cmds(fm, "umount")) >= 3
            await cl.wait_for(gone, timeout=10)
            assert not any(t.endswith(("/data", "/ceph", "/gl")) for t in fm.mounts)
    run(main(), timeout=60)


def test_block_plugins_attach_format_and_detach(run):
    async def main():
        async with LocalCluster(nodes=1, gpus_per_node=0) as cl:
            c = cl.client
            fm = FakeMounter()
            cl.nodes[0].kubelet.volumes.mounter = fm
            iqn = "iqn.2026-10.io.kamd:data"
            dev = f"/dev/disk/by-path/ip-10.2.0.1:3260-iscsi-{iqn}-lun-3"
            fm.appear[("iscsiadm", "-m", "node", "-p", "10.2.0.1:3260")] = dev
            fm.results[("blkid", "-p", "-s", "TYPE", "-s", "PTTYPE", "-o", "export", dev)] = (2, "")   # blank
            fm.results[("rbd", "map")] = (0, "/dev/rbd0\n")
            fm.results[("blkid", "-p", "-s", "TYPE", "-s", "PTTYPE", "-o", "export", "/dev/rbd0")] = (0, "TYPE=xfs\n")
            fm.devices.add("/dev/disk/by-path/pci-0000:41:00.0-fc-0x500a0981891b8dc5-lun-1")
            fm.results[("blkid", "-p", "-s", "TYPE", "-s", "PTTYPE", "-o", "export",
                        "/dev/disk/by-path/pci-0000:41:00.0-fc-0x500a0981891b8dc5-lun-1")] = (0, "PTTYPE=gpt\n")
            await c.create("secrets", {"metadata": {"name": "rbd", "namespace": "default"},
                                       "data": {"key": base64.b64encode(b"rbdkey").decode()}})
            vols = [{"name": "scratch", "iscsi": {"targetPortal": "10.2.0.1", "iqn": iqn, "lun": 3, "fsType": "ext4"}},
                    {"name": "rbdv", "rbd": {"monitors": ["10.3.0.1:6789"], "image": "img", "pool": "kube",
                                             "user": "kube", "secretRef": {"name": "rbd"}, "fsType": "xfs"}}]
            await c.create("pods", _pod("blk", vols))
            await cl.wait_pod("blk")
            log = fm.log
            idx = lambda pred: next(i for i, c in enumerate(log) if pred(c))  # noqa: E731
            disc = idx(lambda c: c[:3] == ["iscsiadm", "-m", "discoverydb"] and "--discover" in c)
            login = idx(lambda c: c[:3] == ["iscsiadm", "-m", "node"] and "--login" in c)
            mkfs = idx(lambda c: c[0] == "mkfs.ext4")
            mnt = idx(lambda c: c[0] == "mount" and c[-2] == dev)
            assert disc < login < mkfs < mnt and log[mkfs] == ["mkfs.ext4", "-F", "-m0", dev]
            rbd = next(c for c in log if c[:2] == ["rbd", "map"])
            assert rbd[2:] == ["kube/img", "--id", "kube", "-m", "10.3.0.1:6789", "--key=rbdkey"]
            assert not any(c[0] == "mkfs.xfs" for c in log)                  # already formatted
            assert any(c[0] == "mount" and c[-2] == "/dev/rbd0" and c[2] == "xfs" for c in log)
            # an FC LUN with a partition table and no file system is refused, never formatted
            await c.create("pods", _pod("fc", [{"name": "lun", "fc": {"targetWWNs": ["500A0981891B8DC5"], "lun": 1}}]))
            await asyncio.sleep(1.0)
            p = await c.get("pods", "fc", "default")
            assert p["status"].get("phase") != "Running"
            assert not any(c[0].startswith("mkfs") and "fc-0x" in c[-1] for c in log)
            # deletion: unmount, then iSCSI logout and rbd unmap
            await c.delete("pods", "blk", "default", grace_period=0)

            async def detached():
                return any("--logout" in c for c in log) and any(c[:2] == ["rbd", "unmap"] for c in log)
            await cl.wait_for(detached, timeout=10)
            assert log.index(next(c for c in log if "--logout" in c)) > log.index(
                next(c for c in log if c[0] == "umount" and c[-1].endswith("/scratch")))
    run(main(), timeout=60)


def test_format_and_mount_never_formats_readonly_or_partitioned(run, tmp_path):
    async def main():
        fm = FakeMounter()
        ctx = PluginContext(None, "default", fm, str(tmp_path))
        fm.results[("blkid",)] = (2, "")
        await format_and_mount(ctx, "/dev/sdz", str(tmp_path / "ro"), "ext4", read_only=True)
        assert not any(c[0].startswith("mkfs") for c in fm.log)
        fm.results[("blkid",)] = (0, "PTTYPE=dos\n")
        try:
            await format_and_mount(ctx, "/dev/sdy", str(tmp_path / "pt"), "ext4", read_only=False)
            raise AssertionError("a partitioned device must not be mounted/formatted")
        except Exception as e:  # noqa: BLE001
            assert "partition table" in str(e)
    run(main())


def test_pod_dir_removal_skips_mount_points(tmp_path):
    d = tmp_path / "pod" / "volumes"
    (d / "nfs-live").mkdir(parents=True)
    (d / "nfs-live" / "remote-file").write_text("precious")
    (d / "local").mkdir()
    (d / "local" / "f").write_text("x")
    fm = FakeMounter()
    fm.mounts[str(d / "nfs-live")] = ("nas:/x", [])
    _rmtree_no_mounts(str(tmp_path / "pod"), fm)
    assert (d / "nfs-live" / "remote-file").read_text() == "precious"
    assert not os.path.exists(d / "local")
