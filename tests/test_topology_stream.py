"""Fragmentation regression for the mixed-size GPU pod stream (kubemark/topology_stream.py).

Pins, on a fixed seed, what the bench's `topology_stream` secondary reports for the real
8xMI355X node shape (one fully connected hive, 2 NUMA nodes) and for CPX partitions, against
the reference's placement (spreading priorities + first-N devices) on the same stream.
"""
from kubernetes_amd.kubemark import topology_stream as ts


def test_node_devices_are_the_real_plugin_shape():
    from kubernetes_amd.api import core
    spx = ts.node_devices("SPX")
    cpx = ts.node_devices("CPX")
    assert len(spx) == 8 and len(cpx) == 64
    a = [d["attributes"] for d in spx.values()]
    assert len({x[core.ATTR_HIVE] for x in a}) == 1                   # one fully connected hive
    assert sorted(x[core.ATTR_NUMA] for x in a) == ["0"] * 4 + ["1"] * 4
    assert all(int(x[core.ATTR_XGMI_PEERS], 16) == 0xFF for x in a)
    assert len({d["attributes"][core.ATTR_SOCKET] for d in cpx.values()}) == 8


def test_stream_fragmentation_is_pinned():
    r = ts.run(n_nodes=16, n_pods=2000, seed=1, load=0.85)
    spx, cpx = r["spx"], r["cpx"]
    for s in (spx, cpx):
        assert s["never_placed"] == 0
        # a node with enough free devices always yields a valid set (fully connected hive)
        assert s["node_frag_blocked_fraction"] == 0.0
        # multi-GPU pods wait less while the capacity exists but is spread over nodes
        assert s["frag_wait_s_per_multi_pod"] <= 0.6 * s["reference_frag_wait_s_per_multi_pod"]
        assert s["frag_blocked_fraction"] <= s["reference_frag_blocked_fraction"]
        assert s["wait_p99_s"] <= s["reference_wait_p99_s"]
        assert 0.7 <= s["utilization"] <= 0.95
    # 2/4-GPU sets inside one NUMA node far more often than first-N placement
    assert spx["numa_fit_fraction"] >= spx["reference_numa_fit_fraction"] + 0.15
    assert spx["numa_fit_fraction"] >= 0.55
    # CPX: 8/16-partition pods on the fewest packages almost always, first-N almost never
    assert cpx["min_packages_fraction"] >= 0.6 and cpx["reference_min_packages_fraction"] <= 0.2
