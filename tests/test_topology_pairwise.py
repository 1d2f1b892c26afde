"""Pairwise xGMI connectivity in placement ("fully connected (all pairs XGMI link
type, from amdsmi_topo_get_link_type)").

The reference allocator takes the first N devices in map order with no topology
(`plugin/pkg/scheduler/core/extended_resources.go:113-150`). Here the plugin publishes each
package's hive index and the bitmask of hive peers it reaches over an up xGMI link, and the
scheduler places an N-GPU set on a clique of that graph. Fixture: one 8-GPU hive whose 2<->5
link is down (both report 6/7 links) — with a per-device link COUNT only, {2, 5, ...} would
pass the "each has >= N-1 links" test.
"""
import asyncio
from itertools import combinations

from kubernetes_amd.api import core
from kubernetes_amd.cluster import LocalCluster
from kubernetes_amd.deviceplugin.amdgpu import gpu_attributes, xgmi_peer_map
from kubernetes_amd.native import amdsmi
from kubernetes_amd.scheduler import topology


def _devs(links_down=((2, 5),), hives=1):
    smi = amdsmi.SMI(fixture=amdsmi.fixture_file(8, hives=hives, links_down=links_down))
    gpus = smi.gpus()
    peers = xgmi_peer_map(smi, gpus)
    return {g.device_id_str: {"id": g.device_id_str, "health": core.HEALTHY,
                              "attributes": gpu_attributes(g, smi.metrics(g.index), peers[g.index])} for g in gpus}


class _ER:
    """The scheduler cache's per-node ERManager view the allocator reads."""
    def __init__(self, devs):
        self.available = {core.AMD_GPU: dict(devs)}
        self.hive_free = {core.AMD_GPU: {}}
        for i, d in devs.items():
            self.hive_free[core.AMD_GPU].setdefault(d["attributes"][core.ATTR_HIVE], {})[i] = d
        self.nfree = {core.AMD_GPU: len(devs)}

    def take(self, ids):
        for i in ids:
            d = self.available[core.AMD_GPU].pop(i)
            del self.hive_free[core.AMD_GPU][d["attributes"][core.ATTR_HIVE]][i]
        self.nfree[core.AMD_GPU] -= len(ids)


def _idx(devs, ids):
    return {int(devs[i]["attributes"][core.ATTR_XGMI_NODE]) for i in ids}


def test_peer_attributes_from_link_table():
    devs = _devs()
    by_node = {int(d["attributes"][core.ATTR_XGMI_NODE]): d["attributes"] for d in devs.values()}
    assert by_node[2][core.ATTR_XGMI_PEERS] == f"{0xff & ~(1 << 5):x}"
    assert by_node[5][core.ATTR_XGMI_PEERS] == f"{0xff & ~(1 << 2):x}"
    assert by_node[0][core.ATTR_XGMI_PEERS] == "ff"
    assert by_node[2][core.ATTR_XGMI_LINKS] == "6" and by_node[5][core.ATTR_XGMI_LINKS] == "6"


def test_allocator_never_pairs_unlinked_packages():
    """Fill the hive with 2-GPU pods: {2, 5} must never be a pair, every pair is linked."""
    devs = _devs()
    er = _ER(devs)
    pairs = []
    for _ in range(4):
        req = [topology.Request("g", core.AMD_GPU, 2, None)]
        ok, _, why = topology.feasible(req, er, topology.REQUIRED)
        b, score, why2 = topology.allocate(req, er, topology.REQUIRED)
        assert ok == (b is not None), (why, why2)
        if b is None:
            break
        ids = b["g"]["resources"]
        pairs.append(_idx(devs, ids))
        er.take(ids)
    assert pairs and {2, 5} not in pairs, pairs
    assert len(pairs) == 4   # 0-1, 2-3, 4-5... a perfect matching avoiding 2-5 exists


def test_four_gpu_sets_are_cliques():
    devs = _devs(links_down=((2, 5), (1, 6)))
    er = _ER(devs)
    for _ in range(2):
        req = [topology.Request("g", core.AMD_GPU, 4, None)]
        b, _, why = topology.allocate(req, er, topology.REQUIRED)
        if b is None:
            break
        s = _idx(devs, b["g"]["resources"])
        assert {2, 5} - s or not {2, 5} <= s
        assert not {1, 6} <= s
        er.take(b["g"]["resources"])


def test_feasible_agrees_with_allocate_when_no_clique_is_left():
    """Only {2, 5} free: two devices, but not linked — a required 2-GPU pod does not fit."""
    devs = _devs()
    keep = {i for i, d in devs.items() if d["attributes"][core.ATTR_XGMI_NODE] in ("2", "5")}
    er = _ER({i: d for i, d in devs.items() if i in keep})
    req = [topology.Request("g", core.AMD_GPU, 2, None)]
    ok, _, why = topology.feasible(req, er, topology.REQUIRED)
    b, _, why2 = topology.allocate(req, er, topology.REQUIRED)
    assert not ok and b is None and "xGMI" in why and "xGMI" in why2
    # preferred policy may still span (low score), as for spanning hives
    ok, score, _ = topology.feasible(req, er, topology.PREFERRED)
    assert ok and score == 1.0


def test_full_hive_pod_is_unschedulable_with_a_down_link():
    """An 8-GPU pod needs every pair linked: a hive with a down link cannot host it."""
    devs = _devs()
    er = _ER(devs)
    b, _, why = topology.allocate([topology.Request("g", core.AMD_GPU, 8, None)], er, topology.REQUIRED)
    assert b is None
    assert topology.allocate([topology.Request("g", core.AMD_GPU, 8, None)], _ER(_devs(links_down=())),
                             topology.REQUIRED)[0] is not None


def test_end_to_end_four_gpu_pods_avoid_the_broken_pair(run):
    async def main():
        async with LocalCluster(nodes=1, gpus_per_node=8, links_down=((2, 5),)) as cl:
            c = cl.client
            node = await c.get("nodes", "node-0")
            devs = node["status"]["extendedResources"][core.AMD_GPU]["resources"]
            for k in range(2):
                await c.create("pods", {"metadata": {"name": f"q{k}", "namespace": "default",
                                                     "annotations": {topology.POLICY_ANNOTATION: topology.REQUIRED}},
                                        "spec": {"containers": [{"name": "c", "image": "x",
                                                                 "resources": {"limits": {core.AMD_GPU: "4"}}}]}})
            sets = []
            for k in range(2):
                p = await cl.wait_pod(f"q{k}", timeout=20)
                sets.append(_idx(devs, p["spec"]["extendedResources"][0]["assigned"]))
            for s in sets:
                assert not {2, 5} <= s, sets
                peers = {int(d["attributes"][core.ATTR_XGMI_NODE]): int(d["attributes"][core.ATTR_XGMI_PEERS], 16)
                         for d in devs.values()}
                assert all((peers[a] >> b) & 1 for a, b in combinations(s, 2)), s
    run(main(), timeout=60)


def test_runtime_link_failure_updates_peers(run):
    """A link that fails after registration: the plugin's health poll republishes the peer masks."""
    async def main():
        async with LocalCluster(nodes=1, gpus_per_node=8) as cl:
            plugin = cl.nodes[0].plugin
            plugin.smi.fake_set_link(0, 7, xgmi=False)
            try:
                assert plugin.poll_health()
                await asyncio.sleep(0.3)

                async def republished():
                    n = await cl.client.get("nodes", "node-0")
                    ds = n["status"]["extendedResources"][core.AMD_GPU]["resources"].values()
                    a = {int(d["attributes"][core.ATTR_XGMI_NODE]): d["attributes"][core.ATTR_XGMI_PEERS] for d in ds}
                    return a if a[0] == "7f" and a[7] == "fe" else None
                await cl.wait_for(republished, 10)
            finally:
                plugin.smi.fake_set_link(0, 7, xgmi=True)
    run(main(), timeout=60)


def test_link_probe_prunes_weak_links_from_peer_map(run, tmp_path):
    """A link the SMI reports up but that measures far below a healthy xGMI link (p2p copy)
    leaves the published link graph; the slowest peer copy is published per device."""
    from kubernetes_amd.deviceplugin.amdgpu import ATTR_XGMI_P2P_GBPS, AMDGPUPlugin
    from kubernetes_amd.deviceplugin.linkprobe import ProbeResult, parse
    from kubernetes_amd.native import amdsmi

    def probe(hips):
        pairs = {(a, b): 60.0 for a in hips for b in hips if a != b}
        pairs[(1, 2)] = 3.5                     # degraded link, one direction is enough
        return ProbeResult(pairs, {h: 2500.0 for h in hips})

    async def main():
        smi = amdsmi.SMI(fixture=amdsmi.fixture_file(8))
        p = AMDGPUPlugin(str(tmp_path), smi=smi, health_interval=0, link_probe=probe, link_min_gbps=25)
        before = dict(p.peers)
        weak = await p.run_link_probe()
        assert weak == {frozenset((1, 2))}
        g = {x.index: x for x in smi.gpus()}
        l1, l2 = p.peers[1][0], p.peers[2][0]
        assert not (p.peers[1][1] >> l2) & 1 and not (p.peers[2][1] >> l1) & 1
        assert (before[1][1] >> l2) & 1                                  # it was there before
        assert p.peers[0] == before[0]
        attrs = {d.ID: dict(d.Attributes) for d in p.devices}
        assert attrs[g[1].device_id_str][ATTR_XGMI_P2P_GBPS] == "3"
        assert attrs[g[0].device_id_str][ATTR_XGMI_P2P_GBPS] == "60"
    run(main())
    # the native probe's JSON
    r = parse('{"mode": "p2p", "devices": 2, "bytes": 1, "local": [{"dev": 0, "GBps": 2400.0}, '
              '{"dev": 1, "GBps": 2390.5}], "pairs": [{"src": 0, "dst": 1, "peer": true, "GBps": 51.2}, '
              '{"src": 1, "dst": 0, "peer": true, "GBps": 50.9}]}', [4, 6])
    assert r.pairs == {(4, 6): 51.2, (6, 4): 50.9} and r.local == {4: 2400.0, 6: 2390.5}
