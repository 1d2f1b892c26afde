"""KubeletConfiguration files and Dynamic Kubelet Config (node.spec.configSource → ConfigMap →
checkpoint → validate → apply or keep last-known-good; KubeletConfigOk condition).
Reference: pkg/kubelet/kubeletconfig/controller.go, apis/kubeletconfig/validation."""
import os

import pytest

from kubernetes_amd.cluster import LocalCluster
from kubernetes_amd.kubelet import kubeletconfig as kc


def test_load_validate_defaults():
    cfg = kc.load("kind: KubeletConfiguration\napiVersion: kubeletconfig/v1alpha1\nmaxPods: 64\n"
                  "nodeStatusUpdateFrequency: 1m30s\nevictionHard: {memory.available: 1Gi}\n")
    assert cfg["maxPods"] == 64 and cfg["imageGCHighThresholdPercent"] == 85
    kw = kc.to_kwargs(cfg)
    assert kw["pods"] == 64 and kw["node_status_update_frequency"] == 90.0 and kw["eviction_hard"] == "memory.available<1Gi"
    for bad in ("imageGCHighThresholdPercent: 120", "imageGCLowThresholdPercent: 90\nimageGCHighThresholdPercent: 80",
                "nodeStatusUpdateFrequency: 0s", "cpuManagerPolicy: dynamic", "kind: Pod"):
        with pytest.raises(kc.ConfigError):
            kc.load(bad)
    assert kc.parse_duration("250ms") == 0.25 and kc.parse_duration("1h2m3s") == 3723


def test_dynamic_kubelet_config(run, tmp_path):
    async def main():
        cl = LocalCluster(nodes=1, gpus_per_node=0, workdir=str(tmp_path / "c"),
                          kubelet_kwargs={"dynamic_config_dir": str(tmp_path / "dyn"),
                                          "node_status_update_frequency": 0.2})
        await cl.start()
        c = cl.client
        try:
            good = await c.create("configmaps", {"metadata": {"name": "kcfg-1"}, "data": {
                "kubelet": "kind: KubeletConfiguration\nmaxPods: 42\nnodeStatusUpdateFrequency: 200ms\n"}}, "kube-system")
            await c.patch("nodes", "node-0", {"spec": {"configSource": {"configMapRef": {
                "name": "kcfg-1", "namespace": "kube-system", "uid": good["metadata"]["uid"]}}}})

            def cond(n):
                return next((x for x in n["status"]["conditions"] if x["type"] == "KubeletConfigOk"), {})

            async def applied():
                n = await c.get("nodes", "node-0")
                return n if n["status"]["capacity"]["pods"] == "42" and cond(n).get("status") == "True" else None
            n = await cl.wait_for(applied, 15)
            assert "using current" in cond(n)["message"]
            assert os.path.exists(tmp_path / "dyn" / "checkpoints" / good["metadata"]["uid"] / "kubelet")
            assert kc.startup_checkpoint(str(tmp_path / "dyn"))["maxPods"] == 42     # restart would use it

            bad = await c.create("configmaps", {"metadata": {"name": "kcfg-2"}, "data": {
                "kubelet": "kind: KubeletConfiguration\nimageGCHighThresholdPercent: 150\n"}}, "kube-system")
            await c.patch("nodes", "node-0", {"spec": {"configSource": {"configMapRef": {
                "name": "kcfg-2", "namespace": "kube-system", "uid": bad["metadata"]["uid"]}}}})

            async def rejected():
                n = await c.get("nodes", "node-0")
                return n if cond(n).get("status") == "False" else None
            n = await cl.wait_for(rejected, 15)
            assert "last-known-good" in cond(n)["message"] and n["status"]["capacity"]["pods"] == "42"
            assert kc.startup_checkpoint(str(tmp_path / "dyn"))["maxPods"] == 42     # falls back to LKG

            await c.patch("nodes", "node-0", {"spec": {"configSource": None}})

            async def local():
                n = await c.get("nodes", "node-0")
                return n if n["status"]["capacity"]["pods"] == "110" and cond(n).get("status") == "True" else None
            await cl.wait_for(local, 15)
        finally:
            await cl.stop()
    run(main(), timeout=60)
