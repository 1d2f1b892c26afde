"""The e2e conformance specs against an in-process cluster (process runtime, all controllers),
the way test/e2e runs against a real cluster; the GPU spec is skipped on CPU and runs in the GPU
tier (tests/test_gpu_e2e.py)."""
from kubernetes_amd.cluster import LocalCluster
from kubernetes_amd.e2e import specs  # noqa: F401
from kubernetes_amd.e2e.framework import SPECS, run_specs


def test_conformance_specs_pass(run, tmp_path):
    async def main():
        cl = LocalCluster(nodes=2, gpus_per_node=0, runtime="process", workdir=str(tmp_path / "c"),
                          controllers=["*"], kubelet_http=True)
        await cl.start()
        try:
            lines = []
            res = await run_specs(cl.url, focus="Conformance", timeout=90, out=lines.append)
        finally:
            await cl.stop()
        failed = [r for r in res if not r.ok]
        assert len(res) >= 20 and not failed, "\n".join(r.name + ": " + r.error for r in failed)
    run(main(), timeout=300)
    assert any("Feature:GPU" in t for _, _, tags in SPECS for t in tags)
