"""amd-smi Prometheus exporter (DCGM-exporter replacement) and the Grafana dashboard."""
import json
import os

from kubernetes_amd.cluster import LocalCluster
from kubernetes_amd.client.http import HTTPClient
from kubernetes_amd.monitoring.exporter import AMDSMIExporter
from kubernetes_amd.native import amdsmi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_exporter_metrics_and_pod_attribution(run):
    async def main():
        async with LocalCluster(nodes=1, gpus_per_node=8) as cl:
            await cl.client.create("pods", {"metadata": {"name": "train"}, "spec": {"containers": [
                {"name": "c", "image": "x", "resources": {"limits": {"amd.com/gpu": "2"}}}]}})
            pod = await cl.wait_pod("train")
            kl = cl.nodes[0].kubelet

            async def pods():
                return [s.pod for s in kl.pods.values()]
            cl.smi.fake_set_ecc(6, 2)
            ex = AMDSMIExporter(cl.smi, "node-0", pods_fn=pods)
            port = await ex.start("127.0.0.1", 0)
            c = HTTPClient(f"http://127.0.0.1:{port}")
            st, body = await c.request("GET", "/metrics")
            await c.close()
            await ex.stop()
            cl.smi.fake_set_ecc(6, 0)
            text = body.decode()
            assert st == 200
            assert text.count("amd_gpu_vram_total_bytes{") == 8
            assert 'product="MI355X"' in text and 'arch="gfx950"' in text
            assert "amd_gpu_ecc_uncorrectable_total{gpu=\"6\"" in text
            healthy = [ln for ln in text.splitlines() if ln.startswith("amd_gpu_healthy{")]
            assert sum(ln.endswith(" 0") for ln in healthy) == 1
            alloc = [ln for ln in text.splitlines() if ln.startswith("amd_gpu_pod_allocated{")]
            assert len(alloc) == 2 and all('pod="train"' in ln for ln in alloc)
            for did in pod["spec"]["extendedResources"][0]["assigned"]:
                assert any(did in ln for ln in alloc)
    run(main())


def test_grafana_dashboard_queries_exporter_metrics():
    d = json.load(open(os.path.join(ROOT, "deploy", "monitoring", "grafana-dashboard-mi355x.json")))
    exprs = " ".join(t["expr"] for p in d["panels"] for t in p.get("targets", []))
    for m in ("amd_gpu_gfx_activity_percent", "amd_gpu_vram_used_bytes", "amd_gpu_power_watts",
              "amd_gpu_ecc_uncorrectable_total", "amd_gpu_xgmi_links_up", "amd_gpu_pod_allocated",
              "kubelet_device_plugin_alloc_latency_microseconds"):
        assert m in exprs, m


def _deepest(pid):
    import psutil
    p = psutil.Process(pid)
    while p.children():
        p = p.children()[0]
    return p.pid


def test_per_container_gpu_memory_attribution(run):
    """AMD SMI's per-process list joined with the runtime's container processes: each pod is
    charged its own processes' VRAM (cAdvisor's NVML collector reported the whole device's,
    vendor/github.com/google/cadvisor/accelerators/nvidia.go:172-222); the exporter republishes
    it as amd_gpu_pod_vram_bytes{pod,namespace,container,gpu}."""
    from kubernetes_amd.api import core
    from kubernetes_amd.kubelet import stats

    async def main():
        async with LocalCluster(nodes=1, gpus_per_node=8, runtime="process") as cl:
            for name in ("a", "b"):
                await cl.client.create("pods", {"metadata": {"name": name}, "spec": {"containers": [
                    {"name": "c", "image": "busybox", "command": ["sleep", "30"],
                     "resources": {"limits": {core.AMD_GPU: "1"}}}]}})
            pods = {n: await cl.wait_pod(n, timeout=20) for n in ("a", "b")}
            kl = cl.nodes[0].kubelet
            rt = kl.runtime
            devs = (await cl.client.get("nodes", "node-0"))["status"]["extendedResources"][core.AMD_GPU]["resources"]
            idx = {n: int(devs[p["spec"]["extendedResources"][0]["assigned"][0]]["attributes"][core.ATTR_INDEX])
                   for n, p in pods.items()}
            cid = {n: kl.pods[p["metadata"]["uid"]].containers["c"] for n, p in pods.items()}
            pid = {n: _deepest(rt.meta[cid[n]]["proc"].pid) for n in pods}
            # pod a: 1 GiB on its GPU; pod b: 512 MiB on its own; a host process on b's GPU too
            cl.smi.fake_set_procs(idx["a"], [(pid["a"], "train", 1 << 30, 0)])
            cl.smi.fake_set_procs(idx["b"], [(pid["b"], "serve", 512 << 20, 0), (1, "host-daemon", 7 << 30, 0)])
            try:
                s = stats.summary(kl)
                used = {p["podRef"]["name"]: p["containers"][0]["accelerators"][0]["memoryUsed"] for p in s["pods"]}
                assert used == {"a": 1 << 30, "b": 512 << 20}, used
                ex = AMDSMIExporter(cl.smi, "node-0", stats_fn=lambda: _coro(stats.summary(kl)))
                text = await ex.collect()
                rows = [ln for ln in text.splitlines() if ln.startswith("amd_gpu_pod_vram_bytes{")]
                assert any('pod="a"' in r and r.endswith(f" {1 << 30}") for r in rows), rows
                assert any('pod="b"' in r and r.endswith(f" {512 << 20}") for r in rows), rows
            finally:
                cl.smi.fake_set_procs(idx["a"], [])
                cl.smi.fake_set_procs(idx["b"], [])
    run(main(), timeout=60)


async def _coro(v):
    return v
