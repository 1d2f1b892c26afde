"""Real MI355X end-to-end (GPU box only)."""
import pytest

pytestmark = pytest.mark.gpu


def test_real_gpu_pod_runs_hip_vector_add(run):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from kubernetes_amd.e2e.smoke import gpu_pod_e2e
    r = run(gpu_pod_e2e(), timeout=300)
    print(r)
    assert r["attributes"]["amd.com/arch"].startswith("gfx950")
    assert int(r["attributes"]["amd.com/memory"]) > 250_000
    kfd = [d for d in r["allow"] if d.get("type") == "c" and d.get("allow")]
    assert len(kfd) >= 2


def test_real_gpu_pod_over_cri(run):
    """Same GPU pod, kubelet -> CRI gRPC (kamd-cri, process runtime) -> hip-vector-add on the MI355X."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from kubernetes_amd.e2e.smoke import gpu_pod_e2e
    r = run(gpu_pod_e2e(cri=True), timeout=300)
    assert r["runtime"] == "kamd-process"
    assert "Test PASSED" in r["log"]


def test_real_plugin_capacity_and_health(run):
    import asyncio
    from kubernetes_amd.cluster import LocalCluster

    async def main():
        async with LocalCluster(nodes=1, gpus_per_node=8, real_gpus=True, health_interval=0.5) as cl:
            node = await cl.client.get("nodes", cl.nodes[0].name)
            assert int(node["status"]["capacity"]["amd.com/gpu"]) >= 1
            await asyncio.sleep(1.2)   # a health poll on the real backend keeps devices Healthy
            devs = node["status"]["extendedResources"]["amd.com/gpu"]["resources"]
            assert all(d["health"] == "Healthy" for d in devs.values())
    run(main(), timeout=120)


@pytest.mark.gpu
def test_e2e_gpu_spec_on_real_mi355x(run):
    """The e2e framework's [Feature:GPU] spec (mirror of test/e2e/scheduling/nvidia-gpus.go)
    against a one-node cluster on the real MI355X: two pods get distinct GPUs and both print
    'Test PASSED' from the HIP vector add."""
    from kubernetes_amd.cluster import LocalCluster
    from kubernetes_amd.e2e import specs  # noqa: F401
    from kubernetes_amd.e2e.framework import run_specs

    async def main():
        async with LocalCluster(nodes=1, gpus_per_node=8, runtime="process", real_gpus=True, kubelet_http=True) as cl:
            res = await run_specs(cl.url, focus="Feature:GPU", timeout=150)
        # the [Feature:MultiGPU] spec skips on a box with fewer than 4 GPUs
        ran = [r for r in res if not r.skipped]
        assert ran and all(r.ok for r in res), [(r.name, r.error) for r in res]
    run(main(), timeout=200)


def test_burn_in_gates_real_gpus_then_pod_runs(run):
    """The plugin's acceptance test on the real MI355X: HIP vector_add exact, MFMA bf16 GEMM
    8192^3 within tolerance and >= 700 TFLOP/s, the fp8 block-scaled MFMA GEMM >= 1400 TFLOP/s,
    HBM copy >= 3000 GB/s; only then does the GPU
    turn Healthy, carry its measured numbers, and take a pod."""
    import asyncio
    from kubernetes_amd.api import core
    from kubernetes_amd.cluster import LocalCluster
    from kubernetes_amd.deviceplugin.burnin import BurnIn

    async def main():
        async with LocalCluster(nodes=1, gpus_per_node=8, real_gpus=True, burn_in=BurnIn()) as cl:
            plugin = cl.nodes[0].plugin
            loop = asyncio.get_running_loop()
            end = loop.time() + 90
            while loop.time() < end and len(plugin._burn) < len(plugin.gpus):
                await asyncio.sleep(0.2)
            for i, r in plugin._burn.items():
                print(i, r)
            passed = {i: r for i, r in plugin._burn.items() if r.ok}
            assert passed, plugin._burn
            for r in passed.values():
                assert r.tflops >= 700 and r.hbm_gbps >= 3000 and r.mfma_rel_err < 1e-2 and r.vadd_err == 0
                assert r.fp8_tflops >= 1400 and r.fp8_rel_err < 1e-2
            await asyncio.sleep(0.5)
            node = await cl.client.get("nodes", cl.nodes[0].name)
            devs = node["status"]["extendedResources"][core.AMD_GPU]["resources"]
            for i in passed:
                assert devs[i]["health"] == "Healthy" and devs[i]["attributes"]["amd.com/burn-in"] == "passed"
                assert int(devs[i]["attributes"]["amd.com/mfma-tflops"]) >= 700
            await cl.client.create("pods", {"metadata": {"name": "after-burn-in"}, "spec": {"containers": [
                {"name": "c", "image": "kubernetes-amd/hip-vector-add", "resources": {"limits": {core.AMD_GPU: "1"}}}]}})
            p = await cl.wait_pod("after-burn-in", timeout=30)
            assert p["spec"]["extendedResources"][0]["assigned"][0] in passed
    run(main(), timeout=150)


def test_pod_vram_attribution_on_mi355x(run):
    """A pod holding 1 GiB of HBM shows up with ~1 GiB in the kubelet summary API: AMD SMI's
    process list (amdsmi_get_gpu_process_list) joined with the pod's container process."""
    import asyncio
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from kubernetes_amd.api import core
    from kubernetes_amd.cluster import LocalCluster
    from kubernetes_amd.kubelet import stats

    async def main():
        async with LocalCluster(nodes=1, gpus_per_node=8, runtime="process", real_gpus=True) as cl:
            await cl.client.create("pods", {"metadata": {"name": "hold"}, "spec": {"restartPolicy": "Never", "containers": [
                {"name": "c", "image": "kubernetes-amd/hip-vector-add", "args": ["--hold-mib", "1024", "--hold-seconds", "30"],
                 "resources": {"limits": {core.AMD_GPU: "1"}}}]}})
            p = await cl.wait_pod("hold", timeout=60)
            kl = cl.nodes[0].kubelet
            cid = kl.pods[p["metadata"]["uid"]].containers["c"]
            log_path = kl.runtime.container_status(cid).log_path

            async def holding():
                return "HOLDING" in open(log_path).read()
            await cl.wait_for(holding, 30, 0.1)
            used = 0
            for _ in range(50):
                s = stats.summary(kl)
                acc = [c["accelerators"][0] for q in s["pods"] for c in q["containers"] if c.get("accelerators")]
                used = acc[0]["memoryUsed"] if acc else 0
                if used >= 1 << 30:
                    break
                await asyncio.sleep(0.2)
            print("memoryUsed", used, "deviceMemoryUsed", acc[0].get("deviceMemoryUsed") if acc else None)
            assert (1 << 30) <= used <= (2 << 30), (used, acc)
            await cl.client.delete("pods", "hold", "default")
    run(main(), timeout=150)


def test_xgmi_link_probe_on_mi355x(run, tmp_path):
    """`xgmi-probe --p2p` on the box's GPUs: local copy bandwidth of an HBM3E device, one JSON
    object; the plugin's link probe over the real SMI publishes no weak link."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from kubernetes_amd.deviceplugin.amdgpu import AMDGPUPlugin
    from kubernetes_amd.deviceplugin.linkprobe import run_probe
    from kubernetes_amd.native import amdsmi
    smi = amdsmi.SMI()
    hips = sorted(g.hip_id if g.hip_id >= 0 else g.index for g in smi.gpus())
    r = run_probe(hips, mib=256, iters=10)
    print(r.local, r.pairs)
    assert not r.error, r.error
    assert set(r.local) == set(hips) and all(v > 500 for v in r.local.values())
    assert len(r.pairs) == len(hips) * (len(hips) - 1)

    async def main():
        p = AMDGPUPlugin(str(tmp_path), smi=smi, health_interval=0, link_probe=run_probe)
        assert await p.run_link_probe() == set()
    run(main(), timeout=120)
