"""Checkpoints: checksummed store, CRI pod-sandbox checkpoints surviving a runtime restart
(NOTREADY until removed), kubelet bootstrap-pod checkpoints run without the API server.
Reference: dockershim/docker_checkpoint_test.go, kubelet/checkpoint/checkpoint_test.go."""
import asyncio
import json
import os

import pytest

from kubernetes_amd.client.rest import Client
from kubernetes_amd.cluster import LocalCluster
from kubernetes_amd.cri import api as A
from kubernetes_amd.cri.remote import RemoteRuntime
from kubernetes_amd.cri.server import CRIServer
from kubernetes_amd.kubelet.kubelet import Kubelet
from kubernetes_amd.kubelet.runtime.stub import StubRuntime
from kubernetes_amd.utils.checkpoint import CheckpointManager, CorruptCheckpoint


def test_checkpoint_store(tmp_path):
    cm = CheckpointManager(str(tmp_path / "ck"))
    cm.create("a", {"version": "v1", "x": [1, 2]})
    assert cm.get("a") == {"version": "v1", "x": [1, 2]}
    p = tmp_path / "ck" / "a"
    d = json.loads(p.read_text())
    d["x"] = [9]
    p.write_text(json.dumps(d))
    with pytest.raises(CorruptCheckpoint):
        cm.get("a")
    cm.create("b", {"v": 1})
    assert [k for k, _ in cm.load_all()] == ["b"] and not p.exists()      # corrupt ones are dropped
    with pytest.raises(ValueError):
        cm.create("../escape", {})


def test_cri_sandbox_checkpoints_survive_restart(run, tmp_path):
    async def main():
        sock, ck = str(tmp_path / "cri.sock"), str(tmp_path / "sandbox")
        srv = await CRIServer(StubRuntime(), sock, checkpoint_dir=ck).start()
        rt = await RemoteRuntime(sock, relist_period=0).connect()
        pod = {"metadata": {"name": "p", "namespace": "ml", "uid": "uid-p"}, "spec": {}}
        sid = await rt.run_pod_sandbox(pod, {})
        assert len(os.listdir(ck)) == 1
        await rt.close()
        await srv.stop()
        srv2 = await CRIServer(StubRuntime(), sock, checkpoint_dir=ck).start()      # runtime restarted
        try:
            lst = await srv2.ListPodSandbox(A.MSG["ListPodSandboxRequest"](), None)
            assert [(x.id, x.state, x.metadata.name, x.metadata.namespace) for x in lst.items] == \
                [(sid, A.SANDBOX_NOTREADY, "p", "ml")]
            await srv2.StopPodSandbox(A.MSG["StopPodSandboxRequest"](pod_sandbox_id=sid), None)
            await srv2.RemovePodSandbox(A.MSG["RemovePodSandboxRequest"](pod_sandbox_id=sid), None)
            assert os.listdir(ck) == []
            assert not (await srv2.ListPodSandbox(A.MSG["ListPodSandboxRequest"](), None)).items
        finally:
            await srv2.stop()
    run(main())


def test_bootstrap_pod_checkpoints(run, tmp_path):
    ck = str(tmp_path / "bootstrap")

    async def main():
        cl = LocalCluster(nodes=1, gpus_per_node=0, workdir=str(tmp_path / "c"),
                          kubelet_kwargs={"bootstrap_checkpoint_path": ck})
        await cl.start()
        c = cl.client
        try:
            await c.create("pods", {"metadata": {"name": "apiserver", "annotations": {
                "node.kubernetes.io/bootstrap-checkpoint": "true"}}, "spec": {"containers": [
                    {"name": "c", "image": "kube-apiserver"}]}}, "kube-system")
            await c.create("pods", {"metadata": {"name": "plain"}, "spec": {"containers": [
                {"name": "c", "image": "x"}]}}, "default")

            async def written():
                return len(os.listdir(ck)) == 1
            await cl.wait_for(written, 10)
        finally:
            await cl.stop()
        # "reboot": a fresh kubelet whose API server is unreachable runs the checkpointed pod
        rt = StubRuntime()
        kl = Kubelet(Client("http://127.0.0.1:9", timeout=0.2), "node-0", rt, emit_events=False,
                     root_dir=str(tmp_path / "kl2"), bootstrap_checkpoint_path=ck)
        assert kl._restore_checkpointed_pods() == 1
        for _ in range(100):
            if any(s.pod["metadata"]["name"] == "apiserver" and s.sandbox for s in kl.pods.values()):
                break
            await asyncio.sleep(0.02)
        st = next(s for s in kl.pods.values() if s.pod["metadata"]["name"] == "apiserver")
        assert st.sandbox and st.containers.get("c")
        for t in list(kl._workers.values()):
            t.cancel()
    run(main(), timeout=60)
