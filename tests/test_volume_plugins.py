"""FlexVolume (exec driver protocol: init / mount <dir> <json> / unmount <dir>) and gitRepo
volumes, through a real kubelet + process runtime. Reference: pkg/volume/flexvolume
(driver-call.go, flexvolume_test.go), pkg/volume/git_repo."""
import json
import os
import stat
import subprocess
import sys

from kubernetes_amd.cluster import LocalCluster

FLEX = r'''#!{py}
import json, os, sys
log = os.environ.get("FLEX_LOG") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "calls.log")
with open(log, "a") as f:
    f.write(json.dumps(sys.argv[1:]) + "\n")
cmd = sys.argv[1]
if cmd == "init":
    print(json.dumps({{"status": "Success", "capabilities": {{"attach": False}}}}))
elif cmd == "mount":
    target, opts = sys.argv[2], json.loads(sys.argv[3])
    os.makedirs(target, exist_ok=True)
    with open(os.path.join(target, "dataset.txt"), "w") as f:
        f.write(opts.get("dataset", "") + ":" + opts["kubernetes.io/pod.name"])
    print(json.dumps({{"status": "Success"}}))
elif cmd == "unmount":
    p = os.path.join(sys.argv[2], "dataset.txt")
    if os.path.exists(p):
        os.unlink(p)
    print(json.dumps({{"status": "Success"}}))
else:
    print(json.dumps({{"status": "Not supported"}}))
'''


def test_flexvolume_and_git_repo(run, tmp_path):
    plugdir = tmp_path / "flex"
    drv = plugdir / "amd.com~nvme" / "nvme"
    drv.parent.mkdir(parents=True)
    drv.write_text(FLEX.format(py=sys.executable))
    drv.chmod(drv.stat().st_mode | stat.S_IEXEC)
    repo = tmp_path / "models"
    repo.mkdir()
    git = ["git", "-c", "user.email=t@t", "-c", "user.name=t"]
    subprocess.run(["git", "init", "-q"], cwd=repo, check=True)
    (repo / "config.json").write_text('{"layers": 61}')
    subprocess.run(git + ["add", "."], cwd=repo, check=True)
    subprocess.run(git + ["commit", "-q", "-m", "v1"], cwd=repo, check=True)
    rev = subprocess.run(["git", "rev-parse", "HEAD"], cwd=repo, check=True, capture_output=True, text=True).stdout.strip()
    (repo / "config.json").write_text('{"layers": 62}')
    subprocess.run(git + ["commit", "-q", "-am", "v2"], cwd=repo, check=True)

    async def main():
        cl = LocalCluster(nodes=1, gpus_per_node=0, runtime="process", workdir=str(tmp_path / "c"),
                          kubelet_kwargs={"volume_plugin_dir": str(plugdir)})
        await cl.start()
        c = cl.client
        kl = cl.nodes[0].kubelet
        try:
            await c.create("pods", {"metadata": {"name": "trainer"}, "spec": {
                "containers": [{"name": "c", "image": "busybox", "command": ["sh", "-c", "sleep 30"],
                                "volumeMounts": [{"name": "scratch", "mountPath": "/scratch"},
                                                 {"name": "code", "mountPath": "/code"}]}],
                "volumes": [{"name": "scratch", "flexVolume": {"driver": "amd.com/nvme", "fsType": "xfs",
                                                              "options": {"dataset": "imagenet"}}},
                            {"name": "code", "gitRepo": {"repository": str(repo), "revision": rev,
                                                         "directory": "."}}]}}, "default")

            async def running():
                p = await c.get("pods", "trainer", "default")
                return p if (p.get("status") or {}).get("phase") == "Running" else None
            p = await cl.wait_for(running, 30)
            st = next(s for s in kl.pods.values() if s.pod["metadata"]["name"] == "trainer")
            with open(os.path.join(st.volumes["scratch"], "dataset.txt")) as f:
                assert f.read() == "imagenet:trainer"
            with open(os.path.join(st.volumes["code"], "config.json")) as f:
                assert json.load(f)["layers"] == 61            # checked out at the pinned revision
            calls = [json.loads(x) for x in (drv.parent / "calls.log").read_text().splitlines()]
            assert calls[0] == ["init"] and calls[1][0] == "mount"
            opts = json.loads(calls[1][2])
            assert opts["kubernetes.io/fsType"] == "xfs" and opts["kubernetes.io/readwrite"] == "rw"
            assert opts["kubernetes.io/pod.uid"] == p["metadata"]["uid"]
            await c.delete("pods", "trainer", "default", grace_period=0)

            async def unmounted():
                cs = [json.loads(x) for x in (drv.parent / "calls.log").read_text().splitlines()]
                return any(x[0] == "unmount" for x in cs)
            await cl.wait_for(unmounted, 20)
        finally:
            await cl.stop()
    run(main(), timeout=90)


def test_fs_group_ownership_never_follows_symlinks(tmp_path):
    """the fsGroup walk changes entries through O_PATH|O_NOFOLLOW descriptors, so a
    symlink a container planted in its volume never makes the kubelet chmod the target."""
    import os
    import stat
    from kubernetes_amd.kubelet.volumes import set_volume_ownership
    outside = tmp_path / "host-secret"
    outside.write_text("x")
    os.chmod(outside, 0o600)
    vol = tmp_path / "vol"
    (vol / "sub").mkdir(parents=True)
    (vol / "sub" / "f").write_text("y")
    os.chmod(vol / "sub" / "f", 0o600)
    os.symlink(outside, vol / "sub" / "link")
    set_volume_ownership(str(vol), os.getgid(), readonly=False)
    assert stat.S_IMODE(os.stat(outside).st_mode) == 0o600          # untouched
    assert stat.S_IMODE(os.stat(vol / "sub" / "f").st_mode) == 0o660
    d = os.stat(vol / "sub").st_mode
    assert d & stat.S_ISGID and d & 0o010
