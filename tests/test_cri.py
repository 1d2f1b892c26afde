"""CRI over gRPC: server (dockershim role) + remote runtime client (kubelet side) + PLEG relist,
image service / image manager / image GC, streaming exec and port-forward.

Parity: `pkg/kubelet/apis/cri/testing/fake_runtime_service.go`-style round trips,
`pkg/kubelet/pleg/generic_test.go` (relist emits ContainerDied), `pkg/kubelet/images/*_test.go`.
"""
import asyncio
import os
import sys

import pytest

from kubernetes_amd.cri import api as A
from kubernetes_amd.cri.remote import RemoteRuntime
from kubernetes_amd.cri.server import CRIServer, ImageStore, LocalImageService, stub_image_resolver
from kubernetes_amd.kubelet.images import ImageGCError, ImageGCManager, ImageManager, ImagePullError, default_pull_policy
from kubernetes_amd.kubelet.runtime.base import EXITED, RUNNING, RunContainerOptions, RuntimeError_
from kubernetes_amd.kubelet.runtime.process import ProcessRuntime
from kubernetes_amd.kubelet.runtime.stub import StubRuntime


def pod(name="p", uid="uid-1", ann=None):
    return {"metadata": {"name": name, "namespace": "default", "uid": uid, "labels": {"app": "x"},
                         "annotations": dict(ann or {})}, "spec": {"containers": []}}


def test_messages_roundtrip_field_numbers():
    cfg = A.MSG["ContainerConfig"](metadata=A.MSG["ContainerMetadata"](name="c", attempt=2),
                                   devices=[A.MSG["Device"](container_path="/dev/kfd", host_path="/dev/kfd", permissions="rw")])
    raw = cfg.SerializeToString()
    # field 1 (metadata, length-delimited) first, then field 8 (devices) = tag 0x42
    assert raw[0] == 0x0a and b"\x42" in raw
    assert A.MSG["ContainerConfig"].FromString(raw) == cfg
    assert len(A.RUNTIME_METHODS) == 21 and len(A.IMAGE_METHODS) == 5


@pytest.mark.parametrize("server_t,client_t", [("lite", "lite"), ("grpc", "lite"), ("lite", "grpc")])
def test_remote_runtime_over_stub(run, tmp_path, server_t, client_t):
    # CRI over utils/grpclite by default; each side also interoperates with a grpc-core peer
    async def main():
        sock = str(tmp_path / "cri.sock")
        srv = await CRIServer(StubRuntime(), sock, transport=server_t).start()
        rt = await RemoteRuntime(sock, relist_period=0.05, transport=client_t).connect()
        exits = []
        rt.on_exit(lambda uid, cid: exits.append((uid, cid)))
        try:
            assert (await rt.version())["runtimeName"] == "kamd-stub"
            p = pod(ann={"kubemark.amd.com/run-seconds": "0.1"})
            sid = await rt.run_pod_sandbox(p, {"amd.com/gpu-ids": "0,1"})
            lst = await srv.ListPodSandbox(A.MSG["ListPodSandboxRequest"](), None)
            assert lst.items[0].labels[A.POD_UID] == "uid-1"
            assert lst.items[0].annotations["amd.com/gpu-ids"] == "0,1"
            opts = RunContainerOptions(envs=[{"name": "AMD_VISIBLE_DEVICES", "value": "0"}],
                                       devices=[{"pathOnHost": "/dev/dri/renderD128", "pathInContainer": "/dev/dri/renderD128",
                                                 "permissions": "rw"}])
            cid = await rt.create_container(sid, p, {"name": "c", "image": "img:1", "env": [{"name": "A", "value": "1"}]}, opts)
            # the backend runtime saw the original container spec and the device options
            meta = srv.rt.meta[cid]
            assert meta["container"]["env"] == [{"name": "A", "value": "1"}]
            assert meta["opts"].devices[0]["pathOnHost"] == "/dev/dri/renderD128"
            assert meta["opts"].envs == [{"name": "AMD_VISIBLE_DEVICES", "value": "0"}]
            await rt.start_container(cid)
            assert rt.container_status(cid).state == RUNNING
            for _ in range(100):           # the container exits after 0.1 s; PLEG relist sees it
                if exits:
                    break
                await asyncio.sleep(0.02)
            assert exits == [("uid-1", cid)]
            assert rt.container_status(cid).state == EXITED and rt.relists > 0
            rc, _ = await rt.exec_sync(cid, ["true"], 1)
            assert rc == 126            # not running
            await rt.stop_pod_sandbox(sid)
            await rt.remove_pod_sandbox(sid)
            assert rt.container_status(cid) is None
            assert (await rt.status()) == {"RuntimeReady": True, "NetworkReady": True}
        finally:
            await rt.close()
            await srv.stop()
    run(main())


def test_remote_process_runtime_exec_logs_stats(run, tmp_path):
    async def main():
        sock = str(tmp_path / "cri.sock")
        srv = await CRIServer(ProcessRuntime(str(tmp_path / "rt")), sock).start()
        rt = await RemoteRuntime(sock, relist_period=0.05).connect()
        sid = None
        try:
            p = pod()
            sid = await rt.run_pod_sandbox(p, {})
            code = "import sys,time; print('hello-from-container', flush=True); time.sleep(30)"
            cid = await rt.create_container(sid, p, {"name": "c", "image": "busybox", "command": [sys.executable, "-c", code]},
                                            RunContainerOptions())
            await rt.start_container(cid)
            for _ in range(100):
                if b"hello-from-container" in await rt.container_logs(cid):
                    break
                await asyncio.sleep(0.05)
            assert b"hello-from-container" in await rt.container_logs(cid)
            rc, out = await rt.exec_sync(cid, ["sh", "-c", "echo exec-ok; exit 3"], 5)
            assert rc == 3 and b"exec-ok" in out
            # streaming exec through the CRI streaming server URL
            url = await rt.exec_url(cid, ["sh", "-c", "echo streamed"])
            from kubernetes_amd.cri.streaming import read_exec_stream
            rc, out = await read_exec_stream(url)
            assert rc == 0 and out == b"streamed\n"
            stats = await rt.container_stats()
            assert stats[cid]["working_set_bytes"] > 0
            await rt.stop_container(cid, 1)
            assert rt.container_status(cid).state == EXITED
        finally:
            if sid is not None:       # the sandbox (pause) outlives the CRI server by design
                await rt.stop_pod_sandbox(sid)
                await rt.remove_pod_sandbox(sid)
            await rt.close()
            await srv.stop()
    run(main())


def test_streaming_port_forward(run, tmp_path):
    async def main():
        async def echo(r, w):
            data = await r.read(100)
            w.write(b"echo:" + data)
            await w.drain()
            w.close()
        backend = await asyncio.start_server(echo, "127.0.0.1", 0)
        port = backend.sockets[0].getsockname()[1]
        sock = str(tmp_path / "cri.sock")
        srv = await CRIServer(StubRuntime(), sock).start()
        rt = await RemoteRuntime(sock, relist_period=0).connect()
        try:
            sid = await rt.run_pod_sandbox(pod(), {})
            url = await rt.port_forward_url(sid, [port])
            from kubernetes_amd.cri.streaming import open_port_forward
            r, w = await open_port_forward(url, port)
            w.write(b"ping")
            await w.drain()
            assert await r.read(100) == b"echo:ping"
            w.close()
            # tokens are single-use
            with pytest.raises(ConnectionError):
                await open_port_forward(url, port)
        finally:
            await rt.close()
            await srv.stop()
            backend.close()
    run(main())


def test_image_service_and_pull_policy(run, tmp_path):
    async def main():
        sock = str(tmp_path / "cri.sock")
        srv = await CRIServer(ProcessRuntime(str(tmp_path / "rt")), sock,
                              image_resolver=lambda ref: 100 if "known" in ref else None).start()
        rt = await RemoteRuntime(sock, relist_period=0).connect()
        try:
            img = rt.images
            assert await img.image_status("known/app:1") is None
            ref = await img.pull_image("known/app:1")
            assert ref.startswith("sha256:")
            assert (await img.image_status("known/app:1"))["repoTags"] == ["known/app:1"]
            assert (await img.image_fs_info())["usedBytes"] == 100
            with pytest.raises(RuntimeError_):
                await img.pull_image("missing/app:1")
            m = ImageManager(img, backoff_initial=5.0)
            assert await m.ensure_image_exists(pod(), {"image": "known/app:1"}) == ref
            with pytest.raises(ImagePullError) as e:
                await m.ensure_image_exists(pod(), {"image": "missing/app:1"})
            assert e.value.reason == "ErrImagePull"
            with pytest.raises(ImagePullError) as e:
                await m.ensure_image_exists(pod(), {"image": "missing/app:1"})
            assert e.value.reason == "ImagePullBackOff" and 0 < m.retry_after("missing/app:1") <= 5.0
            with pytest.raises(ImagePullError) as e:
                await m.ensure_image_exists(pod(), {"image": "known/other:2", "imagePullPolicy": "Never"})
            assert e.value.reason == "ErrImageNeverPull"
            await img.remove_image("known/app:1")
            assert await img.list_images() == []
        finally:
            await rt.close()
            await srv.stop()
    run(main())
    assert default_pull_policy("busybox") == "Always"
    assert default_pull_policy("busybox:latest") == "Always"
    assert default_pull_policy("repo:5000/busybox:1.2") == "IfNotPresent"


def test_image_gc_frees_lru_unused(run):
    async def main():
        store = ImageStore(lambda ref: 30)
        svc = LocalImageService(store)
        for n in ("a:1", "b:1", "c:1", "d:1"):
            await svc.pull_image(n)
        t = [1000.0]
        in_use = {"d:1"}
        gc = ImageGCManager(svc, capacity_bytes=100, in_use=lambda: in_use, high=85, low=50, min_age=10, clock=lambda: t[0])
        await gc.detect(t[0])
        with pytest.raises(ImageGCError, match="but freed 0 bytes"):
            await gc.garbage_collect()                     # all images younger than min_age
        t[0] += 20
        gc.records[store.by_tag["a:1"]]["last"] = 990.0   # a used most recently among the unused ones
        freed = await gc.garbage_collect()                 # fs full (0 available) -> free down to 50% (need 50)
        assert freed == 60                                 # b and c (never used) go first, then it stops
        left = sorted(t for i in store.images.values() for t in i["repo_tags"])
        assert left == ["a:1", "d:1"]                      # in-use image kept, a used more recently
    run(main())


def test_kubelet_on_remote_runtime(run, tmp_path):
    """A real kubelet drives pods through the CRI socket; ErrImageNeverPull surfaces in status."""
    from kubernetes_amd.cluster import LocalCluster

    async def main():
        sock = str(tmp_path / "cri.sock")
        srv = await CRIServer(StubRuntime(), sock).start()
        rt = await RemoteRuntime(sock, relist_period=0.05).connect()
        cl = LocalCluster(nodes=0, gpus_per_node=0)
        await cl.start()
        try:
            h = await cl.add_node("n-cri", runtime=rt)
            c = cl.client
            await c.create("pods", {"metadata": {"name": "ok", "namespace": "default",
                                                 "annotations": {"kubemark.amd.com/run-seconds": "0.2"}},
                                    "spec": {"nodeName": "n-cri", "restartPolicy": "Never",
                                             "containers": [{"name": "c", "image": "img:1"}]}})
            await c.create("pods", {"metadata": {"name": "never", "namespace": "default"},
                                    "spec": {"nodeName": "n-cri", "containers": [
                                        {"name": "c", "image": "absent:1", "imagePullPolicy": "Never"}]}})
            phase = reason = None
            for _ in range(200):
                p = await c.get("pods", "ok", "default")
                q = await c.get("pods", "never", "default")
                phase = (p.get("status") or {}).get("phase")
                cs = ((q.get("status") or {}).get("containerStatuses") or [{}])[0]
                reason = ((cs.get("state") or {}).get("waiting") or {}).get("reason")
                if phase == "Succeeded" and reason == "ErrImageNeverPull":
                    break
                await asyncio.sleep(0.05)
            assert phase == "Succeeded"
            assert reason == "ErrImageNeverPull"
            assert h.kubelet.runtime.runtime_name == "kamd-stub"
        finally:
            await cl.stop()
            await rt.close()
            await srv.stop()
    run(main(), timeout=60)


def test_kubelet_restart_adopts_pods_over_cri(run, tmp_path):
    """kubelet restart with the runtime in its own process (the CRI split): the new kubelet
    lists sandboxes and containers (ListPodSandbox / ListContainers, pod-uid labels) and adopts
    them — same container ids, restart counts kept from the CRI attempt — instead of starting
    the pods again."""
    from kubernetes_amd.cluster import LocalCluster
    from kubernetes_amd.kubelet.devicemanager.manager import ManagerStub
    from kubernetes_amd.kubelet.kubelet import Kubelet
    from kubernetes_amd.client.rest import Client

    async def main():
        sock = str(tmp_path / "cri.sock")
        srv = await CRIServer(StubRuntime(), sock).start()
        rt = await RemoteRuntime(sock, relist_period=0.05).connect()
        cl = LocalCluster(nodes=0, gpus_per_node=0)
        await cl.start()
        rt2 = None
        try:
            h = await cl.add_node("n-cri", runtime=rt)
            c = cl.client
            await c.create("pods", {"metadata": {"name": "keep", "namespace": "default"},
                                    "spec": {"nodeName": "n-cri", "containers": [{"name": "c", "image": "img:1"}]}})
            p = await cl.wait_pod("keep")
            cid = p["status"]["containerStatuses"][0]["containerID"]
            await h.kubelet.stop()
            await rt.close()
            # a new runtime client + kubelet, as after a kubelet process restart
            rt2 = await RemoteRuntime(sock, relist_period=0.05).connect()
            kl2 = Kubelet(Client(cl.url), "n-cri", rt2, ManagerStub(), root_dir=str(tmp_path / "kl2"))
            await kl2.run()
            h.kubelet = kl2
            await cl.wait_for(lambda: asyncio.sleep(0, result=kl2.adopted_pods == 1), timeout=10)
            await asyncio.sleep(0.3)
            p = await c.get("pods", "keep", "default")
            cs = p["status"]["containerStatuses"][0]
            assert cs["containerID"] == cid and cs["restartCount"] == 0 and p["status"]["phase"] == "Running"
            lst = await srv.rt.pod_states()
            assert sum(len(v["sandboxes"]) for v in lst.values()) == 1     # nothing started twice
            assert sum(len(v["containers"]) for v in lst.values()) == 1
        finally:
            await cl.stop()
            if rt2 is not None:
                await rt2.close()
            await srv.stop()
    run(main(), timeout=60)


def test_run_as_user_over_cri(run, tmp_path):
    """securityContext.runAsUser travels in CRI LinuxContainerSecurityContext and the process
    runtime's container-init takes that identity before exec."""
    import os

    async def main():
        sock = str(tmp_path / "cri.sock")
        srv = await CRIServer(ProcessRuntime(str(tmp_path / "rt")), sock).start()
        rt = await RemoteRuntime(sock, relist_period=0.05).connect()
        uid = 65534 if os.geteuid() == 0 else os.geteuid()
        sid = None
        try:
            p = pod()
            sid = await rt.run_pod_sandbox(p, {})
            cid = await rt.create_container(sid, p, {"name": "c", "image": "busybox", "command": ["sh", "-c", "id -u"]},
                                            RunContainerOptions(run_as_user=uid))
            await rt.start_container(cid)
            for _ in range(100):
                if rt.container_status(cid).state == EXITED:
                    break
                await asyncio.sleep(0.05)
            assert (await rt.container_logs(cid)).strip() == str(uid).encode()
        finally:
            if sid is not None:
                await rt.stop_pod_sandbox(sid)
                await rt.remove_pod_sandbox(sid)
            await rt.close()
            await srv.stop()
    run(main())
