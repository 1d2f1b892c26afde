"""Enforced GPU device isolation in the process runtime (kamd-runc).

The reference relied on docker: dockershim mapped the plugin's DeviceSpecs into
`HostConfig.Resources.Devices` (`pkg/kubelet/dockershim/docker_container.go:164-172`) and the
e2e asserted that pods get distinct GPUs (`test/e2e_node/gpu_device_plugin.go:46-143`). Here the
device plugin serves mknod'd stand-ins for `/dev/kfd` and `/dev/dri/renderD128..135` (char
major 226 like real DRM render nodes, no driver behind them), so the test can tell the three
outcomes apart from inside a pod:
  * allocated node: present in the private /dev, the device cgroup allows it -> open() fails
    only in the (absent) driver: ENXIO/ENODEV;
  * another GPU's node in /dev: absent -> ENOENT;
  * another GPU's node reached through its host path: the device cgroup denies it -> EPERM.
Needs root with namespaces (this CI container); the GPU box runs unprivileged without user
namespaces, which the IsolationUnavailable test covers.
"""
import json
import os
import stat
import subprocess

import pytest

from kubernetes_amd.api import core
from kubernetes_amd.cluster import LocalCluster
from kubernetes_amd.kubelet.runtime import process as proc_rt
from kubernetes_amd.kubelet.runtime.base import RunContainerOptions
from kubernetes_amd.kubelet.runtime.process import ProcessRuntime, runc_features

FEATURES = runc_features()
needs_isolation = pytest.mark.skipif(not FEATURES.get("isolation") or os.geteuid() != 0,
                                     reason=f"namespaces not available here: {FEATURES}")

PROBE = r'''
import errno, os, sys
mine = sorted(os.listdir("/dev/dri"))
print("DRI", ",".join(mine))
print("DEV", ",".join(sorted(os.listdir("/dev"))))
def probe(p):
    try:
        os.close(os.open(p, os.O_RDWR))
        return "OPEN"
    except OSError as e:
        return errno.errorcode.get(e.errno, str(e.errno))
print("MINE", probe("/dev/dri/" + mine[0]))
print("KFD", probe("/dev/kfd"))
for m in range(128, 136):
    n = "renderD%d" % m
    if n not in mine:
        print("OTHER_DEV", probe("/dev/dri/" + n))
        print("OTHER_HOST", probe(os.path.join(sys.argv[1], "dri", n)))
        break
print("PID1", open("/proc/1/cmdline").read().split("\0")[0])
print("HIP", os.environ.get("HIP_VISIBLE_DEVICES", "unset"))
'''


def make_dev_root(d):
    os.makedirs(os.path.join(d, "dri"), exist_ok=True)
    os.mknod(os.path.join(d, "kfd"), stat.S_IFCHR | 0o666, os.makedev(1, 3))   # openable (/dev/null)
    for m in range(128, 136):
        os.mknod(os.path.join(d, "dri", f"renderD{m}"), stat.S_IFCHR | 0o666, os.makedev(226, m))
    return d


def parse(log):
    out = {}
    for line in log.splitlines():
        k, _, v = line.partition(" ")
        out.setdefault(k, v)
    return out


def test_features_json_shape():
    f = runc_features()
    assert {"isolation", "mount_ns", "device_cgroup"} <= set(f) or "namespace_error" in f


@needs_isolation
def test_gpu_pod_sees_only_its_render_node(run, tmp_path):
    dev = make_dev_root(str(tmp_path / "dev"))

    async def main():
        async with LocalCluster(nodes=1, gpus_per_node=8, runtime="process", dev_root=dev, isolation="required") as cl:
            c = cl.client
            node = await c.get("nodes", "node-0")
            conds = {x["type"]: x for x in node["status"]["conditions"]}
            assert conds["IsolationUnavailable"]["status"] == "False", conds
            pods = []
            for i in range(2):
                p = {"metadata": {"name": f"iso{i}", "namespace": "default"},
                     "spec": {"restartPolicy": "Never", "containers": [{
                         "name": "c", "image": "busybox", "command": ["python3", "-c", PROBE, dev],
                         "resources": {"limits": {core.AMD_GPU: "1"}}}]}}
                await c.create("pods", p)
            for i in range(2):
                pods.append(await cl.wait_pod(f"iso{i}", phase="Succeeded", timeout=30))
            rt = cl.nodes[0].runtime
            seen = []
            for cs in rt.list_containers():
                r = parse(open(cs.log_path).read())
                seen.append(r["DRI"])
                # exactly one render node, the allocated one, and only default nodes + kfd + dri
                assert len(r["DRI"].split(",")) == 1, r
                assert set(r["DEV"].split(",")) <= {"dri", "fd", "full", "kfd", "null", "ptmx", "pts", "random", "shm",
                                                   "stderr", "stdin", "stdout", "tty", "urandom", "zero"}, r
                assert r["MINE"] in ("ENXIO", "ENODEV"), r     # cgroup allowed; no DRM driver here
                assert r["KFD"] == "OPEN", r
                assert r["OTHER_DEV"] == "ENOENT", r           # not in the container's /dev
                assert r["OTHER_HOST"] == "EPERM", r           # device cgroup denies the host node
                assert r["HIP"] == "unset", r                  # isolation, not env narrowing
                assert r["PID1"] != "/usr/lib/systemd/systemd"
                iso = json.load(open(os.path.join(os.path.dirname(cs.log_path), "isolation.json")))
                assert iso["mount_ns"] and iso["pid_ns"] and iso["dev"] == "private"
                assert iso["device_cgroup"] in ("bpf", "v1")
            # the two pods got distinct GPUs (gpu_device_plugin.go:46-143)
            assert len(set(seen)) == 2, seen
            assigned = [p["spec"]["extendedResources"][0]["assigned"][0] for p in pods]
            assert len(set(assigned)) == 2
    run(main(), timeout=120)


@needs_isolation
def test_exec_enters_the_container(run, tmp_path):
    dev = make_dev_root(str(tmp_path / "dev"))

    async def main():
        rt = ProcessRuntime(str(tmp_path / "rt"), isolation="required")
        pod = {"metadata": {"name": "p", "namespace": "default", "uid": "u-exec"}, "spec": {}}
        sid = await rt.run_pod_sandbox(pod, {})
        opts = RunContainerOptions(devices=[
            {"pathOnHost": os.path.join(dev, "dri", "renderD130"), "pathInContainer": "/dev/dri/renderD130", "permissions": "rw"}])
        cid = await rt.create_container(sid, pod, {"name": "c", "image": "busybox", "command": ["sleep", "30"]}, opts)
        await rt.start_container(cid)
        try:
            rc, out = await rt.exec_sync(cid, ["sh", "-c", "ls /dev/dri; echo pid=$$; hostname"], 10)
            assert rc == 0, out
            lines = out.decode().split()
            assert lines[0] == "renderD130"
            # the exec'd shell lives in the container's pid namespace (sleep is pid 2 under init)
            assert int(lines[1].split("=")[1]) < 100
            assert lines[2] == "p"            # the sandbox's uts namespace
            # two containers of a pod share the sandbox's ipc namespace
            init = rt.meta[cid]["init_pid"]
            sb = rt.sandboxes[sid]["init_pid"]
            assert os.readlink(f"/proc/{init}/ns/ipc") == os.readlink(f"/proc/{sb}/ns/ipc")
            assert os.readlink(f"/proc/{init}/ns/mnt") != os.readlink("/proc/self/ns/mnt")
        finally:
            await rt.stop_container(cid, 1)
            await rt.remove_pod_sandbox(sid)
    run(main(), timeout=60)


@needs_isolation
def test_stop_reaches_the_entrypoint(run, tmp_path):
    """SIGTERM to the container (the kubelet signals kamd-runc's process group) is forwarded
    to the entrypoint through the container's init; the pid namespace dies with it."""
    async def main():
        rt = ProcessRuntime(str(tmp_path / "rt"), isolation="required")
        pod = {"metadata": {"name": "p", "namespace": "default", "uid": "u-stop"}, "spec": {}}
        sid = await rt.run_pod_sandbox(pod, {})
        script = "trap 'echo got-term; exit 7' TERM; sleep 60 & wait"
        cid = await rt.create_container(sid, pod, {"name": "c", "image": "busybox", "command": ["sh", "-c", script]},
                                        RunContainerOptions())
        await rt.start_container(cid)
        import asyncio
        await asyncio.sleep(0.3)
        init = rt.meta[cid]["init_pid"]
        await rt.stop_container(cid, 5)
        st = rt.container_status(cid)
        assert st.exit_code == 7, (st, open(st.log_path).read())
        assert "got-term" in open(st.log_path).read()
        assert not os.path.exists(f"/proc/{init}")
        await rt.remove_pod_sandbox(sid)
    run(main(), timeout=60)


def test_isolation_unavailable_condition(run, monkeypatch):
    """An unprivileged runtime without user namespaces (the GPU box) reports it on the node."""
    monkeypatch.setitem(proc_rt._FEATURES, "", {"isolation": False, "mount_ns": False, "device_cgroup": "none",
                                                 "namespace_error": "No space left on device"})

    async def main():
        async with LocalCluster(nodes=1, gpus_per_node=2, runtime="process") as cl:
            node = await cl.client.get("nodes", "node-0")
            conds = {x["type"]: x for x in node["status"]["conditions"]}
            assert conds["IsolationUnavailable"]["status"] == "True"
            assert "No space left on device" in conds["IsolationUnavailable"]["message"]
            # auto mode still runs the pod, narrowed by HIP_VISIBLE_DEVICES
            await cl.client.create("pods", {"metadata": {"name": "e", "namespace": "default"},
                                            "spec": {"restartPolicy": "Never", "containers": [{
                                                "name": "c", "image": "busybox",
                                                "command": ["sh", "-c", "echo HIP=$HIP_VISIBLE_DEVICES"],
                                                "resources": {"limits": {core.AMD_GPU: "1"}}}]}})
            await cl.wait_pod("e", phase="Succeeded", timeout=30)
            cs = cl.nodes[0].runtime.list_containers()[0]
            assert "HIP=" in open(cs.log_path).read() and "HIP=-1" not in open(cs.log_path).read()
    run(main(), timeout=90)


def test_required_isolation_refuses_device_containers(run, tmp_path, monkeypatch):
    monkeypatch.setitem(proc_rt._FEATURES, "", {"isolation": False, "namespace_error": "no namespaces"})

    async def main():
        rt = ProcessRuntime(str(tmp_path / "rt"), isolation="required")
        pod = {"metadata": {"name": "p", "namespace": "default", "uid": "u-req"}, "spec": {}}
        sid = await rt.run_pod_sandbox(pod, {})
        opts = RunContainerOptions(devices=[{"pathOnHost": "/dev/null", "pathInContainer": "/dev/dri/renderD128"}])
        with pytest.raises(OSError, match="IsolationUnavailable"):
            await rt.create_container(sid, pod, {"name": "c", "image": "busybox", "command": ["true"]}, opts)
        # a container without devices still runs
        cid = await rt.create_container(sid, pod, {"name": "d", "image": "busybox", "command": ["true"]},
                                        RunContainerOptions())
        await rt.start_container(cid)
        await rt.remove_pod_sandbox(sid)
    run(main(), timeout=60)


def test_device_filter_program_assembles():
    """The BPF device program is generated from the OCI allow list; a deny-all rule last in
    evaluation order must not leave unreachable instructions (the verifier rejects them)."""
    if not FEATURES.get("device_cgroup"):
        pytest.skip("no kamd-runc")
    # `features` loads a program built from the default allow list: success means the
    # generator produced verifier-clean code on this kernel (bpf) or v1 is used
    assert FEATURES["device_cgroup"] in ("bpf", "v1", "none")


def test_oci_spec_security_context():
    from kubernetes_amd.kubelet.runtime import oci
    pod = {"metadata": {"name": "p", "uid": "u"}}
    o = RunContainerOptions(run_as_user=1000, run_as_group=2000, supplemental_groups=[3000, 4000],
                            cap_add=["NET_ADMIN"], cap_drop=["MKNOD"], readonly_rootfs=True, oom_score_adj=-998)
    s = oci.build_spec(pod, {"name": "c", "command": ["x"]}, o, rootfs="/", cgroups_path="/cg/pod/ctr-1",
                       ns_paths={"ipc": "/proc/9/ns/ipc"}, host_network=True)
    assert s["process"]["user"] == {"uid": 1000, "gid": 2000, "additionalGids": [3000, 4000]}
    caps = s["process"]["capabilities"]["bounding"]
    assert "CAP_NET_ADMIN" in caps and "CAP_MKNOD" not in caps and "CAP_SYS_ADMIN" not in caps
    assert s["root"]["readonly"] is True and s["process"]["oomScoreAdj"] == -998
    ns = {n["type"]: n.get("path") for n in s["linux"]["namespaces"]}
    assert ns == {"pid": None, "ipc": "/proc/9/ns/ipc", "uts": None, "mount": None}
    assert s["linux"]["cgroupsPath"] == "/cg/pod/ctr-1"
    assert {m["destination"] for m in s["mounts"]} >= {"/proc", "/dev", "/dev/pts", "/dev/shm", "/sys"}
    p = oci.build_spec(pod, {"name": "c", "command": ["x"]}, RunContainerOptions(privileged=True), rootfs="/")
    assert "/dev" not in {m["destination"] for m in p["mounts"]}
    assert p["linux"]["resources"]["devices"] == [{"allow": True, "access": "rwm"}]
    assert "CAP_SYS_ADMIN" in p["process"]["capabilities"]["bounding"]


def test_kamd_runc_rejects_mismatched_device(tmp_path):
    """A spec device whose host node is not the major:minor the kubelet recorded is refused."""
    if not os.access(proc_rt.KAMD_RUNC, os.X_OK) or not FEATURES.get("isolation"):
        pytest.skip("needs kamd-runc with namespaces")
    b = tmp_path / "b"
    b.mkdir()
    spec = {"process": {"args": ["true"], "env": [], "cwd": "/"}, "root": {"path": "/"},
            "mounts": [{"destination": "/dev", "type": "tmpfs", "source": "tmpfs"}],
            "linux": {"devices": [{"path": "/dev/null", "type": "c", "major": 226, "minor": 128}],
                      "namespaces": [{"type": "mount"}]}}
    (b / "config.json").write_text(json.dumps(spec))
    r = subprocess.run([proc_rt.KAMD_RUNC, "run", "--bundle", str(b)], capture_output=True, text=True, timeout=20)
    assert r.returncode == 126 and "1:3" in r.stderr, r.stderr


@pytest.mark.skipif(not os.access(proc_rt.KAMD_RUNC, os.X_OK) or not FEATURES.get("mount_ns") or os.geteuid() != 0,
                    reason="needs kamd-runc with a mount namespace as root")
def test_image_symlinks_cannot_redirect_mounts_to_the_host(tmp_path):
    """An image whose /dev, a volume mountpoint and a masked path are ABSOLUTE symlinks to host
    paths: every mountpoint, /dev node and /dev/ptmx link must be created inside the rootfs
    (resolved like a chroot, runc's securejoin), never in the host directories."""
    host_dev, host_data, host_etc = (tmp_path / n for n in ("host_dev", "host_data", "host_etc"))
    for d in (host_dev, host_data, host_etc):
        d.mkdir()
    (host_dev / "ptmx").write_text("host file")
    (host_etc / "secret").write_text("host secret")
    rootfs = tmp_path / "b" / "rootfs"
    rootfs.mkdir(parents=True)
    os.symlink(str(host_dev), rootfs / "dev")
    os.symlink(str(host_data), rootfs / "data")
    os.symlink(str(host_etc) + "/../host_etc", rootfs / "etc")
    vol = tmp_path / "vol.txt"
    vol.write_text("volume")
    before = {d: sorted(os.listdir(d)) for d in (host_dev, host_data, host_etc)}
    spec = {"process": {"args": ["/nonexistent"], "env": [], "cwd": "/"}, "root": {"path": "rootfs"},
            "mounts": [{"destination": "/dev", "type": "tmpfs", "source": "tmpfs"},
                       {"destination": "/dev/pts", "type": "devpts", "source": "devpts"},
                       {"destination": "/data/f.txt", "type": "bind", "source": str(vol), "options": ["rbind"]},
                       {"destination": "/data/sub/dir", "type": "tmpfs", "source": "tmpfs"}],
            "linux": {"devices": [], "namespaces": [{"type": "mount"}], "maskedPaths": ["/etc/secret"]}}
    (tmp_path / "b" / "config.json").write_text(json.dumps(spec))
    r = subprocess.run([proc_rt.KAMD_RUNC, "run", "--bundle", str(tmp_path / "b")], capture_output=True,
                       text=True, timeout=20)
    assert r.returncode == 127 and "exec /nonexistent" in r.stderr, r.stderr    # setup finished, then exec failed
    after = {d: sorted(os.listdir(d)) for d in (host_dev, host_data, host_etc)}
    assert after == before
    assert (host_dev / "ptmx").read_text() == "host file"
    # the mountpoints landed inside the rootfs, at the re-rooted symlink targets
    inside = rootfs / str(host_data).lstrip("/")
    assert (inside / "f.txt").exists() and (inside / "sub" / "dir").is_dir()


# -- Landlock tier (unprivileged host without user namespaces) --------------------------------
needs_landlock = pytest.mark.skipif(not FEATURES.get("landlock") or os.geteuid() != 0,
                                    reason=f"Landlock not available here (or not root to set up stand-ins): {FEATURES}")

LL_PROBE = r'''
import errno, os, sys
def probe(p, flags=os.O_RDWR):
    try:
        os.close(os.open(p, flags))
        return "OPEN"
    except OSError as e:
        return errno.errorcode.get(e.errno, str(e.errno))
d = sys.argv[1]
print("LIST", ",".join(sorted(os.listdir(d))))
for n in sorted(os.listdir(d)):
    print("NODE", n, probe(os.path.join(d, n)))
print("ETC", probe("/etc/passwd", os.O_RDONLY))
print("UID", os.getuid())
'''


def _ll_tree(tmp):
    """A world-traversable stand-in for /dev/dri: three char nodes that open like /dev/null."""
    import tempfile
    base = tempfile.mkdtemp(prefix="kamd-ll-", dir="/tmp")
    os.chmod(base, 0o755)
    dri = os.path.join(base, "dri")
    os.makedirs(dri)
    os.chmod(dri, 0o755)
    for m in (128, 129, 130):
        p = os.path.join(dri, f"renderD{m}")
        os.mknod(p, stat.S_IFCHR | 0o666, os.makedev(1, 3))
        os.chmod(p, 0o666)
    return base, dri


def _as_nobody():
    os.setgroups([])
    os.setgid(65534)
    os.setuid(65534)


@needs_landlock
def test_landlock_tier_unprivileged_container(tmp_path):
    """kamd-runc, run as a NON-ROOT uid with no namespaces (the MI355X pool's situation): the
    container can open its allocated stand-in render node and ordinary files, and is refused the
    other nodes of the restricted directory — reported as EPERM through the preloaded errno shim
    (libkamd_devshim.so: Landlock's EACCES would abort ROCr's GPU enumeration), EACCES with the
    shim opted out; `kamd-runc exec --landlock` gives an exec'd process the same ruleset."""
    import shutil
    import sys
    base, dri = _ll_tree(tmp_path)
    # a sibling symlink back to an ancestor (pytest's `pytest-current`): following it would put
    # a rule on the whole tree and void the restriction
    os.symlink(base, os.path.join(base, "current"))
    try:
        b = os.path.join(base, "bundle")
        os.makedirs(b)
        os.chmod(b, 0o777)
        probe = os.path.join(base, "probe.py")
        with open(probe, "w") as f:
            f.write(LL_PROBE)
        os.chmod(probe, 0o644)
        mine = os.path.join(dri, "renderD129")
        # /root is not traversable for nobody: kamd-runc and its errno shim (../lib) move along
        os.makedirs(os.path.join(base, "bin"))
        os.makedirs(os.path.join(base, "lib"))
        runc = os.path.join(base, "bin", "kamd-runc")
        shutil.copy(proc_rt.KAMD_RUNC, runc)
        os.chmod(runc, 0o755)
        shim = os.path.join(base, "lib", "libkamd_devshim.so")
        shutil.copy(os.path.join(os.path.dirname(os.path.dirname(proc_rt.KAMD_RUNC)), "lib", "libkamd_devshim.so"), shim)
        os.chmod(shim, 0o755)
        # the process runtime's default capability list: an unprivileged runc cannot narrow its
        # bounding set and must still start the container (no capability is held anyway)
        caps = ["CAP_CHOWN", "CAP_KILL", "CAP_AUDIT_WRITE"]
        spec = {"process": {"args": [sys.executable, probe, dri], "env": ["PATH=/usr/bin:/bin"], "cwd": "/",
                            "user": {"uid": 65534, "gid": 65534},
                            "capabilities": {k: caps for k in ("bounding", "effective", "permitted")}},
                "root": {"path": "/"}, "mounts": [],
                "annotations": {"kamd.io/isolation-tier": "landlock", "kamd.io/landlock-dir": dri},
                "linux": {"devices": [{"path": mine, "type": "c", "major": 1, "minor": 3}], "namespaces": []}}
        with open(os.path.join(b, "config.json"), "w") as f:
            json.dump(spec, f)
        r = subprocess.run([runc, "run", "--bundle", b], capture_output=True, text=True, timeout=30,
                           preexec_fn=_as_nobody)
        assert r.returncode == 0, r.stderr
        out = r.stdout.splitlines()
        assert "LIST renderD128,renderD129,renderD130" in out              # listing is not restricted
        assert "NODE renderD129 OPEN" in out                              # the allocated node
        assert "NODE renderD128 EPERM" in out and "NODE renderD130 EPERM" in out
        assert "ETC OPEN" in out and "UID 65534" in out
        rep = json.load(open(os.path.join(b, "isolation.json")))
        assert rep["tier"] == "landlock" and rep["landlock_rules"] > 0 and not rep["mount_ns"] and rep["devshim"]
        # opted out of the shim: Landlock's own errno
        spec["annotations"]["kamd.io/devshim"] = "false"
        with open(os.path.join(b, "config.json"), "w") as f:
            json.dump(spec, f)
        r = subprocess.run([runc, "run", "--bundle", b], capture_output=True, text=True, timeout=30,
                           preexec_fn=_as_nobody)
        assert r.returncode == 0, r.stderr
        assert "NODE renderD128 EACCES" in r.stdout.splitlines() and "NODE renderD129 OPEN" in r.stdout.splitlines()
        assert json.load(open(os.path.join(b, "isolation.json")))["devshim"] is False
        # exec into such a container: same restriction for the exec'd process
        target = subprocess.Popen(["sleep", "30"], preexec_fn=_as_nobody)      # "the container" to enter
        try:
            r = subprocess.run([runc, "exec", "--pid", str(target.pid), "--landlock", f"{dri}:{mine}",
                                "--", sys.executable, probe, dri], capture_output=True, text=True, timeout=30,
                               preexec_fn=_as_nobody)
        finally:
            target.kill()
            target.wait()
        assert r.returncode == 0, r.stderr
        assert "NODE renderD129 OPEN" in r.stdout and "NODE renderD130 EPERM" in r.stdout
    finally:
        shutil.rmtree(base, ignore_errors=True)


@needs_landlock
def test_landlock_tier_in_the_process_runtime(run, tmp_path):
    """ProcessRuntime pinned to the Landlock tier: a GPU container (allocated stand-in node)
    runs without namespaces, opens only its node, HIP_VISIBLE_DEVICES is left unset (the tier
    enforces), exec_sync is restricted too, and isolation_status() names the tier."""
    import shutil
    import sys
    base, dri = _ll_tree(tmp_path)
    try:
        rt = ProcessRuntime(str(tmp_path / "rt"), tier="landlock", landlock_dir=dri)
        st = rt.isolation_status()
        assert st["enforced"] and st["tier"] == "landlock" and "landlock" in st["message"]
        probe = os.path.join(base, "probe.py")
        with open(probe, "w") as f:
            f.write(LL_PROBE + 'print("HIP", os.environ.get("HIP_VISIBLE_DEVICES", "unset"))\n')
        pod = {"metadata": {"name": "p", "namespace": "default", "uid": "uid-ll"}, "spec": {}}

        async def main():
            sid = await rt.run_pod_sandbox(pod, {})
            opts = RunContainerOptions(devices=[
                {"pathOnHost": os.path.join(dri, "renderD130"), "pathInContainer": os.path.join(dri, "renderD130"),
                 "permissions": "rw"}])
            cid = await rt.create_container(sid, pod, {"name": "c", "image": "busybox",
                                                       "command": [sys.executable, probe, dri]}, opts)
            await rt.start_container(cid)
            from kubernetes_amd.kubelet.runtime.base import RUNNING
            import asyncio
            for _ in range(200):
                if rt.container_status(cid).state != RUNNING:
                    break
                await asyncio.sleep(0.05)
            log = open(rt.container_status(cid).log_path).read()
            assert "NODE renderD130 OPEN" in log and "NODE renderD128 EPERM" in log, log
            assert "HIP unset" in log
            assert rt.meta[cid]["spec"]["linux"]["namespaces"] == []
            # a long-running container to exec into
            cid2 = await rt.create_container(sid, pod, {"name": "s", "image": "busybox",
                                                        "command": ["sleep", "30"]}, opts)
            await rt.start_container(cid2)
            rc, out = await rt.exec_sync(cid2, [sys.executable, probe, dri], 20)
            assert rc == 0 and b"NODE renderD130 OPEN" in out and b"NODE renderD129 EPERM" in out, out
            await rt.stop_container(cid2, 1)
            await rt.stop_pod_sandbox(sid)
            await rt.remove_pod_sandbox(sid)
        run(main())
    finally:
        shutil.rmtree(base, ignore_errors=True)


def test_tier_selection_and_condition_message(monkeypatch, tmp_path):
    """auto: namespaces when available, else landlock, else none; the IsolationUnavailable
    condition is only raised for tier none."""
    monkeypatch.setitem(proc_rt._FEATURES, "", {"isolation": False, "namespace_error": "ENOSPC", "landlock": 4})
    rt = ProcessRuntime(str(tmp_path / "a"))
    assert rt.tier == "landlock" and rt.isolation_status()["enforced"]
    monkeypatch.setitem(proc_rt._FEATURES, "", {"isolation": False, "namespace_error": "ENOSPC", "landlock": 0,
                                                "landlock_error": "not supported"})
    rt = ProcessRuntime(str(tmp_path / "b"))
    st = rt.isolation_status()
    assert rt.tier == "none" and not st["enforced"] and st["reason"] == "IsolationUnavailable"
    assert "not supported" in st["message"]
    with pytest.raises(ValueError):
        ProcessRuntime(str(tmp_path / "c"), tier="landlock")


@pytest.mark.gpu
def test_landlock_enforced_on_this_host(tmp_path):
    """On the GPU box itself (unprivileged, no user namespaces: the Landlock tier): kamd-runc,
    as this non-root user, confines a container to its allowed entries of a restricted tree.
    Regular files stand in for render nodes (an unprivileged user cannot mknod); Landlock
    checks opens the same way for both. The real /dev/dri of a one-GPU lease holds only the
    allocated node, so this is where denial is shown non-vacuously."""
    import sys
    f = runc_features()
    if f.get("tier") != "landlock":
        pytest.skip(f"this host's tier is {f.get('tier')}, not landlock: {f}")
    base = tmp_path / "ll"
    dri = base / "dri"
    dri.mkdir(parents=True)
    (base / "current").symlink_to(base)       # like pytest-current next to pytest-N
    for n in ("renderD128", "renderD129", "card0"):
        (dri / n).write_text("x")
    probe = base / "probe.py"
    probe.write_text(LL_PROBE)
    b = base / "bundle"
    b.mkdir()
    spec = {"process": {"args": [sys.executable, str(probe), str(dri)], "env": ["PATH=/usr/bin:/bin"], "cwd": "/"},
            "root": {"path": "/"}, "mounts": [],
            "annotations": {"kamd.io/isolation-tier": "landlock", "kamd.io/landlock-dir": str(dri)},
            "linux": {"devices": [{"path": str(dri / "renderD129")}], "namespaces": []}}
    (b / "config.json").write_text(json.dumps(spec))
    r = subprocess.run([proc_rt.KAMD_RUNC, "run", "--bundle", str(b)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert "NODE renderD129 OPEN" in r.stdout, r.stdout
    assert "NODE renderD128 EPERM" in r.stdout and "NODE card0 EPERM" in r.stdout, r.stdout   # via the errno shim
    rep = json.loads((b / "isolation.json").read_text())
    assert rep["tier"] == "landlock" and rep["devshim"]


HSA_PROBE = r'''
import ctypes, glob, json, os, sys
out = {"render_nodes": sorted(os.path.basename(p) for p in glob.glob("/dev/dri/renderD*"))}
opened = {}
for p in out["render_nodes"]:
    try:
        os.close(os.open("/dev/dri/" + p, os.O_RDWR))
        opened[p] = "OPEN"
    except OSError as e:
        opened[p] = __import__("errno").errorcode.get(e.errno, str(e.errno))
out["open"] = opened
lib = None
for cand in ("libhsa-runtime64.so.1", "/opt/rocm/lib/libhsa-runtime64.so.1"):
    try:
        lib = ctypes.CDLL(cand)
        break
    except OSError:
        pass
st = lib.hsa_init()
kinds = []
CB = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_uint64, ctypes.c_void_p)
def cb(agent, data):
    t = ctypes.c_int(-1)
    lib.hsa_agent_get_info(ctypes.c_uint64(agent), 17, ctypes.byref(t))   # HSA_AGENT_INFO_DEVICE
    kinds.append(t.value)
    return 0
keep = CB(cb)
if st == 0:
    lib.hsa_iterate_agents(keep, None)
    lib.hsa_shut_down()
out["hsa_init"] = st
out["gpu_agents"] = kinds.count(1)
out["cpu_agents"] = kinds.count(0)
print("HSA " + json.dumps(out, sort_keys=True))
'''


@pytest.mark.gpu
def test_rocr_start_under_landlock_denial(tmp_path):
    """What the MI355X runtime does when Landlock denies render nodes. Raw Landlock (shim opted
    out) refuses with EACCES, which ROCr's thunk treats as fatal: hsa_init fails with
    HSA_STATUS_ERROR_OUT_OF_RESOURCES (4104) — measured on this pool in round 5. With kamd-runc's
    errno shim (the default) the same denial reads EPERM, as under the device cgroup, and the
    thunk skips the node: HSA starts cleanly with zero GPU agents — what a confined pod on an
    8-GPU node needs for its sibling GPUs — while the allowed node still gives one GPU agent.
    Measured on the box, printed."""
    import sys
    f = runc_features()
    if f.get("tier") != "landlock":
        pytest.skip(f"this host's tier is {f.get('tier')}, not landlock: {f}")
    nodes = sorted(glob_render())
    if not nodes:
        pytest.skip("no /dev/dri/renderD* on this host")
    probe = tmp_path / "hsa_probe.py"
    probe.write_text(HSA_PROBE)
    results = {}
    for label, allowed, shim in (("allowed", [nodes[0]], "true"), ("denied_raw", [], "false"), ("denied", [], "true")):
        b = tmp_path / f"bundle-{label}"
        b.mkdir()
        spec = {"process": {"args": [sys.executable, str(probe)],
                            "env": ["PATH=/usr/bin:/bin", "HSA_ENABLE_IPC_MODE_LEGACY=0"], "cwd": "/"},
                "root": {"path": "/"}, "mounts": [],
                "annotations": {"kamd.io/isolation-tier": "landlock", "kamd.io/landlock-dir": "/dev/dri",
                                "kamd.io/devshim": shim},
                "linux": {"devices": [{"path": p} for p in allowed], "namespaces": []}}
        (b / "config.json").write_text(json.dumps(spec))
        r = subprocess.run([proc_rt.KAMD_RUNC, "run", "--bundle", str(b)], capture_output=True, text=True, timeout=120)
        line = [ln for ln in r.stdout.splitlines() if ln.startswith("HSA ")]
        assert r.returncode == 0 and line, (label, r.returncode, r.stdout[-2000:], r.stderr[-2000:])
        results[label] = json.loads(line[0][4:])
    print("LANDLOCK_ROCR", json.dumps(results, sort_keys=True))
    assert results["allowed"]["hsa_init"] == 0 and results["allowed"]["gpu_agents"] == 1, results
    assert results["denied_raw"]["open"][os.path.basename(nodes[0])] == "EACCES", results
    assert results["denied"]["open"][os.path.basename(nodes[0])] == "EPERM", results
    assert results["denied"]["hsa_init"] == 0 and results["denied"]["gpu_agents"] == 0, results


def glob_render():
    import glob
    return glob.glob("/dev/dri/renderD*")
