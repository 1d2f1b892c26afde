"""Container mounts ported from `pkg/kubelet/kubelet_pods_test.go` (TestMakeMounts,
TestMakeAbsolutePath) with the subPath safety rules (absolute paths, '..', symlinks leaving the
volume) the reference enforces through ValidatePathNoBacksteps / PrepareSafeSubpath."""
import os

import pytest

from kubernetes_amd.kubelet.volumes import VolumeError, make_absolute_path, make_mounts


@pytest.mark.parametrize("inp,out", [("rel/path", "/rel/path"), ("/abs/path", "/abs/path"), ("a", "/a")])
def test_make_absolute_path(inp, out):
    assert make_absolute_path(inp) == out


def test_make_mounts(tmp_path):
    disk, disk4, disk5 = (tmp_path / d for d in ("disk", "disk4", "disk5"))
    for d in (disk, disk4, disk5):
        d.mkdir()
    vols = {"disk": str(disk), "disk4": str(disk4), "disk5": str(disk5)}
    c = {"name": "container1", "volumeMounts": [
        {"mountPath": "/etc/hosts", "name": "disk", "readOnly": False},
        {"mountPath": "/mnt/path3", "name": "disk", "readOnly": True},
        {"mountPath": "/mnt/path4", "name": "disk4", "readOnly": False},
        {"mountPath": "/mnt/path5", "name": "disk5", "readOnly": False}]}
    assert make_mounts(c, vols) == [
        {"containerPath": "/etc/hosts", "hostPath": str(disk), "readOnly": False},
        {"containerPath": "/mnt/path3", "hostPath": str(disk), "readOnly": True},
        {"containerPath": "/mnt/path4", "hostPath": str(disk4), "readOnly": False},
        {"containerPath": "/mnt/path5", "hostPath": str(disk5), "readOnly": False}]


def test_make_mounts_missing_volume():
    with pytest.raises(VolumeError, match='cannot find volume "gone" to mount into container "c"'):
        make_mounts({"name": "c", "volumeMounts": [{"mountPath": "/x", "name": "gone"}]}, {})


def test_subpath_is_created_inside_the_volume_with_its_mode(tmp_path):
    vol = tmp_path / "vol"
    vol.mkdir()
    os.chmod(vol, 0o2775)
    got = make_mounts({"name": "c", "volumeMounts": [{"mountPath": "/data", "name": "v", "subPath": "a/b"}]},
                      {"v": str(vol)})
    assert got[0]["hostPath"] == str(vol / "a" / "b") and (vol / "a" / "b").is_dir()
    assert (os.stat(vol / "a").st_mode & 0o7777) == 0o2775


@pytest.mark.parametrize("sub,err", [
    ("/etc", "must not be an absolute path"),
    ("../escape", "must not contain '..'"),
    ("a/../../escape", "must not contain '..'"),
])
def test_subpath_rejected(tmp_path, sub, err):
    vol = tmp_path / "vol"
    vol.mkdir()
    with pytest.raises(VolumeError, match=err):
        make_mounts({"name": "c", "volumeMounts": [{"mountPath": "/d", "name": "v", "subPath": sub}]}, {"v": str(vol)})


def test_subpath_symlink_escape_refused(tmp_path):
    vol, outside = tmp_path / "vol", tmp_path / "outside"
    vol.mkdir()
    outside.mkdir()
    (vol / "link").symlink_to(outside)                      # a container planted this
    with pytest.raises(VolumeError, match='failed to prepare subPath for volumeMount "v" of container "c"'):
        make_mounts({"name": "c", "volumeMounts": [{"mountPath": "/d", "name": "v", "subPath": "link"}]},
                    {"v": str(vol)})
    with pytest.raises(VolumeError, match="failed to prepare subPath"):
        make_mounts({"name": "c", "volumeMounts": [{"mountPath": "/d", "name": "v", "subPath": "link/new"}]},
                    {"v": str(vol)})
    assert not (outside / "new").exists()
    (vol / "inner").mkdir()
    (vol / "ok").symlink_to(vol / "inner")                  # a link that stays inside is fine
    got = make_mounts({"name": "c", "volumeMounts": [{"mountPath": "/d", "name": "v", "subPath": "ok"}]}, {"v": str(vol)})
    assert got[0]["hostPath"] == str(vol / "inner")
