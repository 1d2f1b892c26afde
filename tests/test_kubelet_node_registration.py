"""Node re-registration reconciliation ported from `pkg/kubelet/kubelet_node_status_test.go`
(TestUpdateDefaultLabels, the controller-managed attach-detach cases of
TestTryRegisterWithApiServer), plus a live kubelet re-registering over an existing Node."""
import pytest

from kubernetes_amd.kubelet.kubelet import (CONTROLLER_MANAGED_ATTACH, DEFAULT_NODE_LABELS, reconcile_cmad_annotation,
                                            update_default_labels)

HOST, ZONE, REGION, ITYPE, OS_, ARCH = DEFAULT_NODE_LABELS


def labels(prefix, extra=None):
    d = {HOST: f"{prefix}-hostname", ZONE: f"{prefix}-zone-failure-domain", REGION: f"{prefix}-zone-region",
         ITYPE: f"{prefix}-instance-type", OS_: f"{prefix}-os", ARCH: f"{prefix}-arch"}
    d.update(extra or {})
    return d


def node(lbls=None, ann=None):
    return {"metadata": {"labels": dict(lbls or {}), "annotations": dict(ann or {})}}


CASES = [
    ("make sure default labels exist", labels("new"), {}, True, labels("new")),
    ("make sure default labels are up to date", labels("new"), labels("old"), True, labels("new")),
    ("make sure existing labels do not get deleted", labels("new"), labels("new", {"please-persist": "foo"}), False,
     labels("new", {"please-persist": "foo"})),
    ("make sure existing labels do not get deleted when initial node has no opinion", {},
     labels("new", {"please-persist": "foo"}), False, labels("new", {"please-persist": "foo"})),
    ("no update needed", labels("new"), labels("new"), False, labels("new")),
    ("not panic when existing node has nil labels", labels("new"), None, True, labels("new")),
    ("an empty opinion removes the label", {HOST: ""}, labels("old"),
     True, {k: v for k, v in labels("old").items() if k != HOST}),
]


@pytest.mark.parametrize("name,initial,existing,needs,final", CASES, ids=[c[0] for c in CASES])
def test_update_default_labels(name, initial, existing, needs, final):
    ex = {"metadata": {}} if existing is None else node(existing)
    assert update_default_labels(node(initial), ex) == needs
    assert ex["metadata"]["labels"] == final


@pytest.mark.parametrize("new,existing,changed,final", [
    ({CONTROLLER_MANAGED_ATTACH: "true"}, {}, True, {CONTROLLER_MANAGED_ATTACH: "true"}),
    ({}, {CONTROLLER_MANAGED_ATTACH: "true"}, True, {}),
    ({CONTROLLER_MANAGED_ATTACH: "true"}, {CONTROLLER_MANAGED_ATTACH: "true"}, False, {CONTROLLER_MANAGED_ATTACH: "true"}),
    ({CONTROLLER_MANAGED_ATTACH: "false"}, {CONTROLLER_MANAGED_ATTACH: "true"}, True, {CONTROLLER_MANAGED_ATTACH: "false"}),
])
def test_reconcile_cmad_annotation(new, existing, changed, final):
    ex = node(ann=existing)
    assert reconcile_cmad_annotation(node(ann=new), ex) == changed
    assert ex["metadata"]["annotations"] == final


def test_kubelet_reregisters_over_existing_node(run):
    from kubernetes_amd.cluster import LocalCluster

    async def main():
        cl = LocalCluster(nodes=0, gpus_per_node=0)
        await cl.start()
        try:
            c = cl.client
            await c.create("nodes", {"metadata": {"name": "n-re", "labels": {HOST: "stale", "team": "a"},
                                                  "annotations": {"keep": "me"}}})
            await cl.add_node("n-re")
            n = await c.get("nodes", "n-re")
            lb, an = n["metadata"]["labels"], n["metadata"]["annotations"]
            assert lb[HOST] == "n-re" and lb["team"] == "a" and lb[OS_] == "linux"
            assert an["keep"] == "me" and an[CONTROLLER_MANAGED_ATTACH] == "true"
            assert any(cd["type"] == "Ready" for cd in n["status"].get("conditions") or ())
        finally:
            await cl.stop()
    run(main(), timeout=60)


def test_too_large_reservation_floors_allocatable_at_zero():
    """`kubelet_node_status_test.go` TestUpdateNewNodeStatusTooLargeReservation: a reservation
    above capacity leaves allocatable 0, never negative."""
    from types import SimpleNamespace

    from kubernetes_amd.kubelet.kubelet import Kubelet
    kl = SimpleNamespace(reserved=({"cpu": "40000m", "memory": "10Gi"}, {}), eviction=None,
                         allocatable_ignore_eviction=True)
    alloc = Kubelet._allocatable(kl, {"cpu": "2", "memory": "1Gi", "pods": "110"})
    assert alloc["cpu"] == "0m" and alloc["memory"] == "0" and alloc["pods"] == "110"
