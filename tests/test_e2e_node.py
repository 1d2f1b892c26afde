"""End-to-end on one node (the reference's `test/e2e_node/gpu_device_plugin.go:46-143` and
BASELINE configs 1-4): plugin registration → node capacity → scheduling with device IDs →
kubelet admission → device injection → pod Running → deletion frees devices."""
import asyncio
import json
import os

import pytest

from kubernetes_amd.api import core
from kubernetes_amd.cluster import LocalCluster


def gpu_pod(name, n=1, cmd=None, image="kubernetes-amd/hip-vector-add", policy="Always", selector=None, ann=None):
    c = {"name": "c", "image": image, "resources": {"limits": {core.AMD_GPU: str(n)}}}
    if cmd:
        c["command"] = cmd
    p = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "namespace": "default", "annotations": ann or {}},
         "spec": {"containers": [c], "restartPolicy": policy}}
    if selector:
        p["spec"]["nodeSelector"] = selector
    return p


def test_node_capacity_and_gpu_pods_stub_runtime(run):
    async def main():
        async with LocalCluster(nodes=1, gpus_per_node=8) as cl:
            c = cl.client
            node = await c.get("nodes", "node-0")
            assert node["status"]["capacity"][core.AMD_GPU] == "8"
            devs = node["status"]["extendedResources"][core.AMD_GPU]["resources"]
            assert len(devs) == 8
            assert node["metadata"]["labels"]["amd.com/gpu.product"] == "MI355X"
            # config 0: CPU-only pod
            await c.create("pods", {"metadata": {"name": "nginx"}, "spec": {"containers": [{"name": "n", "image": "nginx"}]}})
            await cl.wait_pod("nginx")
            # config 3: bin-pack 8 single-GPU pods
            for i in range(8):
                await c.create("pods", gpu_pod(f"g{i}"))
            ids = []
            for i in range(8):
                p = await cl.wait_pod(f"g{i}")
                ids += p["spec"]["extendedResources"][0]["assigned"]
                assert p["status"]["containerStatuses"][0]["ready"]
            assert len(set(ids)) == 8
            # the 9th GPU pod is unschedulable
            await c.create("pods", gpu_pod("g8"))
            await asyncio.sleep(0.3)
            p = await c.get("pods", "g8", "default")
            assert not p["spec"].get("nodeName")
            # delete one -> the pending pod gets the freed device
            freed = (await c.get("pods", "g3", "default"))["spec"]["extendedResources"][0]["assigned"]
            await c.delete("pods", "g3", "default")
            p = await cl.wait_pod("g8", timeout=10)
            assert p["spec"]["extendedResources"][0]["assigned"] == freed
    run(main(), timeout=120)


def test_multi_gpu_hive_and_selector(run):
    async def main():
        async with LocalCluster(nodes=1, gpus_per_node=8, hives=2) as cl:
            c = cl.client
            # config 4: 4-GPU pod lands inside one hive
            await c.create("pods", gpu_pod("four", 4, ann={"amd.com/xgmi-policy": "required"}))
            p = await cl.wait_pod("four")
            node = await c.get("nodes", p["spec"]["nodeName"])
            devs = node["status"]["extendedResources"][core.AMD_GPU]["resources"]
            hives = {devs[i]["attributes"][core.ATTR_HIVE] for i in p["spec"]["extendedResources"][0]["assigned"]}
            assert len(hives) == 1
            # config 5: attribute selector hbm > 256Gi, arch in (gfx950) via explicit extendedResources
            sel = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "sel", "namespace": "default"},
                   "spec": {"containers": [{"name": "c", "image": "x", "extendedResourceRequests": ["gpu"]}],
                            "extendedResources": [{"name": "gpu", "resources": {"limits": {core.AMD_GPU: "2"}},
                                                   "affinity": {"required": [
                                                       {"key": core.ATTR_HBM, "operator": "Gt", "values": ["256Gi"]},
                                                       {"key": core.ATTR_ARCH, "operator": "In", "values": ["gfx950"]}]}}]}}
            await c.create("pods", sel)
            p = await cl.wait_pod("sel")
            assert len(p["spec"]["extendedResources"][0]["assigned"]) == 2
            # unsatisfiable selector stays pending with a FailedScheduling event
            bad = json.loads(json.dumps(sel))
            bad["metadata"]["name"] = "bad"
            bad["spec"]["extendedResources"][0]["affinity"]["required"] = [
                {"key": core.ATTR_ARCH, "operator": "In", "values": ["gfx942"]}]
            await c.create("pods", bad)
            await asyncio.sleep(0.3)
            p = await c.get("pods", "bad", "default")
            assert not p["spec"].get("nodeName")
            cond = core.get_condition(p["status"], core.COND_POD_SCHEDULED)
            assert cond and cond["status"] == "False"
    run(main(), timeout=120)


def test_cpx_partitioned_node_end_to_end(run):
    """A node whose 2 MI355X packages run in CPX mode advertises 16 logical devices; a
    4-partition pod lands on ONE package and its container gets those 4 render nodes."""
    async def main():
        async with LocalCluster(nodes=1, gpus_per_node=2, partition="CPX", runtime="process") as cl:
            c = cl.client
            node = await c.get("nodes", "node-0")
            assert node["status"]["capacity"][core.AMD_GPU] == "16"
            devs = node["status"]["extendedResources"][core.AMD_GPU]["resources"]
            assert {d["attributes"][core.ATTR_PARTITION] for d in devs.values()} == {"CPX"}
            await c.create("pods", gpu_pod("one", 1, cmd=["/bin/sleep", "60"]))
            p1 = await cl.wait_pod("one", timeout=20)
            await c.create("pods", gpu_pod("four", 4, cmd=["/bin/sleep", "60"]))
            p4 = await cl.wait_pod("four", timeout=20)
            a1 = p1["spec"]["extendedResources"][0]["assigned"]
            a4 = p4["spec"]["extendedResources"][0]["assigned"]
            sock = lambda i: devs[i]["attributes"][core.ATTR_SOCKET]   # noqa: E731
            # the 4-partition pod packs into the package the first pod opened (best fit)
            assert len({sock(i) for i in a4}) == 1 and sock(a4[0]) == sock(a1[0]) and not set(a1) & set(a4)
            rt = cl.nodes[0].runtime
            want = sorted(f"renderD{devs[i]['attributes'][core.ATTR_RENDER_MINOR]}" for i in a4)
            specs = []
            for x in rt.list_containers():
                spec = json.load(open(os.path.join(os.path.dirname(x.log_path), "config.json")))
                specs.append(sorted(spec["annotations"]["amd.com/gpu-render-nodes"].split(",")))
            assert want in specs
    run(main(), timeout=120)


def test_process_runtime_injects_devices(run):
    async def main():
        async with LocalCluster(nodes=1, gpus_per_node=2, runtime="process") as cl:
            c = cl.client
            await c.create("pods", gpu_pod("env", 1, cmd=["/bin/sh", "-c", "echo HIP=$HIP_VISIBLE_DEVICES AMD=$AMD_VISIBLE_DEVICES"],
                                           policy="Never"))
            p = await cl.wait_pod("env", phase="Succeeded", timeout=20)
            assert p["status"]["containerStatuses"][0]["state"]["terminated"]["exitCode"] == 0
            rt = cl.nodes[0].runtime
            cs = rt.list_containers()[0]
            log = open(cs.log_path).read()
            idx = p["spec"]["extendedResources"][0]["assigned"]
            assert "HIP=" in log and "AMD=" in log
            spec = json.load(open(os.path.join(os.path.dirname(cs.log_path), "config.json")))
            # /dev/kfd and the render node were requested; on a GPU-less host they are recorded as missing
            ann = spec["annotations"]
            want = {"/dev/kfd"}
            assert want <= set(ann.get("amd.com/missing-device-nodes", "").split(",")) | {d["path"] for d in spec["linux"]["devices"]}
            assert ann["amd.com/gpu-render-nodes"].startswith("renderD")
            del idx
    run(main(), timeout=120)


def test_failing_payload_fails_pod(run):
    async def main():
        async with LocalCluster(nodes=1, gpus_per_node=1, payload=lambda opts: False) as cl:
            await cl.client.create("pods", gpu_pod("bad", 1, policy="Never"))
            p = await cl.wait_pod("bad", phase="Failed", timeout=20)
            assert p["status"]["containerStatuses"][0]["state"]["terminated"]["exitCode"] == 1
    run(main(), timeout=60)


def test_unhealthy_device_reduces_capacity(run):
    async def main():
        async with LocalCluster(nodes=1, gpus_per_node=4) as cl:
            n = cl.nodes[0]
            cl.smi.fake_set_ecc(2, 7)
            assert n.plugin.poll_health()
            for _ in range(200):
                node = await cl.client.get("nodes", n.name)
                if node["status"]["capacity"][core.AMD_GPU] == "3":
                    break
                await asyncio.sleep(0.02)
            assert node["status"]["capacity"][core.AMD_GPU] == "3"
            bad = n.plugin.gpus[2].device_id_str
            assert node["status"]["extendedResources"][core.AMD_GPU]["resources"][bad]["health"] == "Unhealthy"
            for i in range(3):
                await cl.client.create("pods", gpu_pod(f"p{i}"))
            got = []
            for i in range(3):
                got += (await cl.wait_pod(f"p{i}"))["spec"]["extendedResources"][0]["assigned"]
            assert bad not in got
            cl.smi.fake_set_ecc(2, 0)
    run(main(), timeout=60)


def test_container_init_applies_attributes_and_starts(tmp_path):
    """native container-init: cpuset + OOM score applied before exec; unknown binary → 127."""
    import subprocess
    from kubernetes_amd.kubelet.runtime.process import CONTAINER_INIT, _init_argv
    if not os.access(CONTAINER_INIT, os.X_OK):
        pytest.skip("container-init not built")
    cpu = min(os.sched_getaffinity(0))
    argv = _init_argv(["sh", "-c", "cat /proc/self/oom_score_adj; grep Cpus_allowed_list /proc/self/status"],
                      {"PATH": os.environ["PATH"]}, {cpu}, 700, str(tmp_path / "nocgroup"))
    out = subprocess.run(argv, capture_output=True, text=True, check=True).stdout.split()
    assert out[0] == "700" and out[-1] == str(cpu)
    with pytest.raises(FileNotFoundError):
        _init_argv(["no-such-binary-xyz"], {"PATH": "/nonexistent"}, None, 1, None)
    assert subprocess.run([CONTAINER_INIT, "--", "/nonexistent/x"], capture_output=True).returncode == 127


def test_node_density_benchmark_small():
    """e2e_node density/resource-usage equivalent (kubemark/node_density.py) on a tiny config:
    real kubelet process + process runtime, latencies and kubelet CPU/RSS reported."""
    from kubernetes_amd.kubemark import node_density
    out = asyncio.run(node_density.run(batch=3, sequential=2, background=3, monitor=1.0, settle=0.5, period=0.5))
    assert out["batch"]["pods"] == 3 and out["batch"]["all_running_s"] < 25
    assert out["sequential"]["p99_s"] < 10
    assert 0 < out["kubelet_rss_mib"] < 200
    assert out["kubelet_cpu_s_per_pod"] > 0
    assert "steady" in out and out["steady"]["pods"] == 8


def test_node_density_remote_runtime_small():
    """Same benchmark with the kubelet talking CRI to a separate kamd-cri process, whose CPU and
    RSS are reported as the runtime's (the reference's dockershim/docker split)."""
    from kubernetes_amd.kubemark import node_density
    out = asyncio.run(node_density.run(batch=2, sequential=1, background=1, monitor=0.5, settle=0.2, period=0.5,
                                       runtime="remote"))
    assert out["runtime"] == "remote" and out["batch"]["all_running_s"] < 25
    assert 0 < out["runtime_rss_mib"] < 500 and "p95" in out["runtime_cpu_cores"]


def test_gpu_device_plugin_restart_and_plugin_removal(run):
    """The reference's e2e_node GPU device-plugin test (`test/e2e_node/gpu_device_plugin.go:46-143`):
    pods get distinct GPUs; after a kubelet restart the pods keep running with the same
    containers and device assignment (the new kubelet adopts them and re-runs AdmitPod); after
    the device plugin is deleted, GPU capacity drops to 0 and the pods keep running."""
    from kubernetes_amd.client.rest import Client
    from kubernetes_amd.kubelet.devicemanager.manager import ManagerImpl
    from kubernetes_amd.kubelet.kubelet import Kubelet

    async def main():
        async with LocalCluster(nodes=1, gpus_per_node=8) as cl:
            c = cl.client
            h = cl.nodes[0]
            for n in ("gp0", "gp1", "gp2"):
                await c.create("pods", gpu_pod(n, cmd=["sleep", "3600"]))
            before = {}
            for n in ("gp0", "gp1", "gp2"):
                p = await cl.wait_pod(n)
                before[n] = (p["spec"]["extendedResources"][0]["assigned"], p["status"]["containerStatuses"][0]["containerID"])
            assert set(before["gp1"][0]).isdisjoint(before["gp2"][0])
            gone_uid = (await c.get("pods", "gp0", "default"))["metadata"]["uid"]
            # restart the kubelet on the same runtime and plugin directory; gp0 is force-deleted
            # while it is down (its sandbox becomes an orphan the new kubelet removes)
            await h.kubelet.stop()
            await c.delete("pods", "gp0", "default", grace_period=0)
            dm2 = ManagerImpl(h.plugins_dir)
            kl2 = Kubelet(Client(cl.url), h.name, h.runtime, dm2, root_dir=os.path.join(cl.dir, h.name))
            kl2.smi = cl.smi
            kl2.orphan_grace = 0.2
            await kl2.run()
            h.kubelet, h.dm = kl2, dm2
            await cl.wait_for(lambda: asyncio.sleep(0, result=kl2.adopted_pods == 2), timeout=10)
            for n in ("gp1", "gp2"):
                p = await cl.wait_pod(n)
                cs = p["status"]["containerStatuses"][0]
                assert (p["spec"]["extendedResources"][0]["assigned"], cs["containerID"]) == before[n]
                assert cs["restartCount"] == 0 and cs["ready"]
            await cl.wait_for(lambda: asyncio.sleep(0, result=all(
                dm2.pod_resources(kl2.pods[u].pod) is not None for u in kl2.pods)), timeout=10)
            await cl.wait_for(lambda: asyncio.sleep(0, result=not any(
                sb["pod_uid"] == gone_uid for sb in h.runtime.sandboxes.values())), timeout=10)
            # a new pod after the restart still gets a GPU nobody holds
            await c.create("pods", gpu_pod("gp3", cmd=["sleep", "3600"]))
            p3 = await cl.wait_pod("gp3")
            taken = set(before["gp1"][0]) | set(before["gp2"][0])
            assert taken.isdisjoint(p3["spec"]["extendedResources"][0]["assigned"])
            # delete the device plugin: capacity goes to 0, running pods are untouched
            await h.plugin.stop()
            h.plugin = None

            async def zero():
                node = await c.get("nodes", h.name)
                return node["status"]["capacity"].get(core.AMD_GPU) in ("0", None)
            await cl.wait_for(zero, timeout=15)
            for n in ("gp1", "gp2"):
                p = await c.get("pods", n, "default")
                assert p["status"]["phase"] == "Running"
                assert p["status"]["containerStatuses"][0]["containerID"] == before[n][1]
    run(main(), timeout=120)


def test_process_runtime_state_survives_runtime_restart(tmp_path):
    """A new ProcessRuntime on the same root (a restarted kubelet process) re-adopts the live
    sandbox and container from their state.json (pid + kernel start time), watches the adopted
    container's exit through a pidfd, keeps recorded exit codes, and never adopts a dead pid."""
    from kubernetes_amd.kubelet.runtime.base import EXITED, RUNNING, RunContainerOptions
    from kubernetes_amd.kubelet.runtime.process import ProcessRuntime

    async def main():
        pod = {"metadata": {"name": "p", "namespace": "default", "uid": "uid-1234"}, "spec": {}}
        a = ProcessRuntime(str(tmp_path / "rt"))
        sid = await a.run_pod_sandbox(pod, {})
        c1 = await a.create_container(sid, pod, {"name": "long", "command": ["sleep", "30"]}, RunContainerOptions(attempt=2))
        await a.start_container(c1)
        c2 = await a.create_container(sid, pod, {"name": "short", "command": ["sh", "-c", "exit 3"]}, RunContainerOptions())
        await a.start_container(c2)
        for _ in range(200):
            if a.container_status(c2).state == EXITED:
                break
            await asyncio.sleep(0.01)
        b = ProcessRuntime(str(tmp_path / "rt"))                       # "restarted" runtime
        states = await b.pod_states()
        ps = states["uid-1234"]
        assert ps["sandboxes"] == [(sid, True, None)]
        got = {name: (cid, attempt) for name, cid, attempt, _, _ in ps["containers"]}
        assert got["long"] == (c1, 2) and b.container_status(c1).state == RUNNING
        assert b.container_status(c2).state == EXITED and b.container_status(c2).exit_code == 3
        exits = []
        b.on_exit(lambda uid, cid: exits.append(cid))
        await b.stop_container(c1, 1)
        assert b.container_status(c1).state == EXITED
        for _ in range(200):
            if c1 in exits:
                break
            await asyncio.sleep(0.01)
        assert c1 in exits
        await b.remove_pod_sandbox(sid)
        c = ProcessRuntime(str(tmp_path / "rt"))
        assert await c.pod_states() == {}                              # removed state is gone
        await a.remove_pod_sandbox(sid)
    asyncio.run(main())


def test_kubelet_process_restart_keeps_pods_running(tmp_path):
    """A real kubelet process (process runtime) is stopped and started again on the same root
    dir: the pod's container process survives, the new kubelet adopts it (same container id,
    restart count 0), and deleting the pod afterwards still kills it."""
    import signal
    import subprocess
    import sys
    import time as _t
    from kubernetes_amd.client.rest import Client

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=root + os.pathsep + os.environ.get("PYTHONPATH", ""))

    def spawn(args, name):
        return subprocess.Popen([sys.executable, "-m"] + args, env=env, stdout=subprocess.DEVNULL,
                                stderr=open(tmp_path / f"{name}.log", "w"))

    pf = tmp_path / "api.port"
    procs = [spawn(["kubernetes_amd.cmd.apiserver", "--port", "0", "--port-file", str(pf)], "api")]
    kl_args = None
    try:
        t0 = _t.time()
        while not pf.exists():
            assert _t.time() - t0 < 60
            _t.sleep(0.05)
        url = f"http://127.0.0.1:{pf.read_text().strip()}"
        procs.append(spawn(["kubernetes_amd.cmd.scheduler", "--master", url], "sched"))
        kl_args = ["kubernetes_amd.cmd.kubelet", "--api-servers", url, "--hostname-override", "restart-node",
                   "--root-dir", str(tmp_path / "kubelet"), "--container-runtime", "process", "--port", "0",
                   "--container-log-dir", ""]
        kl = spawn(kl_args, "kubelet1")

        async def main():
            nonlocal kl
            c = Client(url)

            async def wait(pred, timeout=30):
                end = _t.time() + timeout
                while _t.time() < end:
                    v = await pred()
                    if v:
                        return v
                    await asyncio.sleep(0.05)
                raise AssertionError("timeout")

            async def running():
                try:
                    p = await c.get("pods", "survivor", "default")
                except Exception:
                    return None
                return p if (p.get("status") or {}).get("phase") == "Running" else None
            await wait(lambda: c.list("nodes"))
            await c.create("pods", {"metadata": {"name": "survivor", "namespace": "default"},
                                    "spec": {"containers": [{"name": "c", "image": "busybox", "command": ["sleep", "300"]}]}})
            p = await wait(running)
            cid = p["status"]["containerStatuses"][0]["containerID"]
            state = json.load(open(tmp_path / "kubelet" / "runtime" / "containers" / cid.split("://")[1] / "state.json"))
            pid = state["pid"]
            kl.send_signal(signal.SIGTERM)
            kl.wait(20)
            os.kill(pid, 0)                                   # the container outlived the kubelet
            kl = spawn(kl_args, "kubelet2")
            await asyncio.sleep(2.0)
            p = await wait(running)
            cs = p["status"]["containerStatuses"][0]
            assert cs["containerID"] == cid and cs["restartCount"] == 0
            os.kill(pid, 0)
            await c.delete("pods", "survivor", "default")

            async def dead():
                try:
                    os.kill(pid, 0)
                except ProcessLookupError:
                    return True
                return False
            await wait(dead)
            await c.close()
        asyncio.run(main())
    finally:
        for p in procs + ([kl] if kl_args else []):
            p.terminate()
        for p in procs + ([kl] if kl_args else []):
            try:
                p.wait(10)
            except subprocess.TimeoutExpired:
                p.kill()
