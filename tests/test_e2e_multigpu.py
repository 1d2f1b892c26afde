"""The [Feature:MultiGPU] e2e spec (a 4-GPU pod with `amd.com/xgmi-policy: required` runs the
`xgmi-probe` RCCL all-reduce, e2e/specs.py:gpu_xgmi_allreduce) on the fake-AMD-SMI fixture —
placement checked, no container process — and its skip below 4 GPUs. The same spec on a real
node with >= 4 MI355X runs the probe (tests/test_gpu_multigpu.py)."""
from kubernetes_amd.cluster import LocalCluster
from kubernetes_amd.e2e import specs  # noqa: F401
from kubernetes_amd.e2e.framework import run_specs


def _run(run, **kw):
    async def main():
        async with LocalCluster(nodes=1, runtime="stub", kubelet_http=True, **kw) as cl:
            return await run_specs(cl.url, focus="Feature:MultiGPU", timeout=60, out=lambda _: None)
    return run(main(), timeout=120)


def test_multigpu_spec_places_a_linked_set_on_the_fixture(run):
    res = _run(run, gpus_per_node=8, hives=2)
    assert len(res) == 1 and res[0].ok and not res[0].skipped, res[0].error


def test_multigpu_spec_skips_below_four_gpus(run):
    res = _run(run, gpus_per_node=2)
    assert len(res) == 1 and res[0].ok and res[0].skipped, res[0].error
    assert "4 healthy" in res[0].error


def test_linked_reads_the_published_peer_bitmask():
    from kubernetes_amd.api import core
    from kubernetes_amd.e2e.specs import _linked

    def dev(node, peers, hive="0x1"):
        return {"attributes": {core.ATTR_HIVE: hive, core.ATTR_XGMI_NODE: str(node), core.ATTR_XGMI_PEERS: peers}}
    full = [dev(i, "ff") for i in range(4)]
    assert _linked(full)
    assert not _linked([dev(0, "fd"), dev(1, "fe")])                              # 0 does not reach 1
    assert not _linked([dev(0, "ff"), dev(1, "ff", hive="0x2")])                  # two hives
