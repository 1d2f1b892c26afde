"""Endpoints controller: `pkg/controller/endpoint/endpoints_controller_test.go` cases over the
fake client — selector-less services left alone, empty selectors select all, ready / notReady
split, the restart-policy exclusions, tolerate-unready, headless services without ports, named
target ports, label propagation, unchanged endpoints not rewritten, deleted services'
endpoints removed, leftover endpoints queued at start."""
import asyncio

import pytest

from kubernetes_amd.client.fake import FakeClient
from kubernetes_amd.client.informer import InformerFactory
from kubernetes_amd.controllers.misc import EndpointsController, repack_subsets, should_pod_be_in_endpoints

NS = "other"


def pods(n, ready=True, start=0, ns=NS, ports=0, restart=None, phase=None):
    out = []
    for i in range(start, start + n):
        p = {"apiVersion": "v1", "kind": "Pod",
             "metadata": {"name": f"pod{i}", "namespace": ns, "uid": f"uid{i}", "labels": {"foo": "bar"},
                          "resourceVersion": "1"},
             "spec": {"containers": [{"name": "c", "ports": [{"name": f"port{j}", "containerPort": 8080 + j}
                                                            for j in range(ports)]}]},
             "status": {"podIP": f"1.2.3.{4 + i}",
                        "conditions": [{"type": "Ready", "status": "True" if ready else "False"}]}}
        if restart:
            p["spec"]["restartPolicy"] = restart
        if phase:
            p["status"]["phase"] = phase
        out.append(p)
    return out


def svc(selector=None, ports=None, ns=NS, name="foo", **spec):
    s = {"apiVersion": "v1", "kind": "Service", "metadata": {"name": name, "namespace": ns},
         "spec": dict(spec, ports=ports if ports is not None else [{"port": 80, "protocol": "TCP",
                                                                    "targetPort": 8080}])}
    if selector is not None:
        s["spec"]["selector"] = selector
    return s


def sync(*objs, key=f"{NS}/foo"):
    async def main():
        c = FakeClient(*objs)
        f = InformerFactory(c)
        ec = EndpointsController(c, f)
        ec.setup()
        f.start()
        await f.wait_for_cache_sync()
        await ec.sync(key)
        writes = [a for a in c.actions if a.verb in ("create", "update", "patch", "delete") and a.resource == "endpoints"]
        try:
            ep = await c.get("endpoints", key.split("/")[1], key.split("/")[0])
        except Exception:      # noqa: BLE001
            ep = None
        return ep, writes
    return asyncio.run(main())


def ips(ss, field="addresses"):
    return [a["ip"] for a in ss.get(field) or ()]


def test_preserve_no_selector():
    ep0 = {"apiVersion": "v1", "kind": "Endpoints", "metadata": {"name": "foo", "namespace": NS},
           "subsets": [{"addresses": [{"ip": "6.7.8.9"}], "ports": [{"port": 1000}]}]}
    ep, writes = sync(svc(None), ep0, *pods(1))
    assert not writes and ep["subsets"] == ep0["subsets"]


def test_new_service_without_pods_creates_empty_endpoints():
    ep, writes = sync(svc({"foo": "bar"}))
    assert [w.verb for w in writes] == ["create"] and ep["subsets"] == []


def test_empty_selector_selects_all_ready_and_not_ready():
    ep, _ = sync(svc({}), *pods(1, ports=1), *pods(1, ready=False, start=1, ports=1))
    assert len(ep["subsets"]) == 1
    ss = ep["subsets"][0]
    assert ips(ss) == ["1.2.3.4"] and ips(ss, "notReadyAddresses") == ["1.2.3.5"]
    assert ss["ports"] == [{"port": 8080, "protocol": "TCP"}]


def test_items_two_ports_and_other_namespace_ignored():
    ports = [{"name": "port0", "port": 80, "protocol": "TCP", "targetPort": 8080},
             {"name": "port1", "port": 88, "protocol": "TCP", "targetPort": 8088}]
    ep, writes = sync(svc({"foo": "bar"}, ports), *pods(3, ports=2), *pods(5, ns="blah", ports=2))
    assert [w.verb for w in writes] == ["create"]
    assert len(ep["subsets"]) == 1 and ips(ep["subsets"][0]) == ["1.2.3.4", "1.2.3.5", "1.2.3.6"]
    assert ep["subsets"][0]["ports"] == [{"name": "port0", "port": 8080, "protocol": "TCP"},
                                         {"name": "port1", "port": 8088, "protocol": "TCP"}]
    tr = ep["subsets"][0]["addresses"][0]["targetRef"]
    assert (tr["kind"], tr["name"], tr["namespace"]) == ("Pod", "pod0", NS)


def test_named_target_port_only_on_pods_that_have_it():
    p = pods(2, ports=0)
    p[0]["spec"]["containers"][0]["ports"] = [{"name": "http", "containerPort": 9376}]
    ep, _ = sync(svc({"foo": "bar"}, [{"port": 80, "targetPort": "http"}]), *p)
    assert len(ep["subsets"]) == 1 and ips(ep["subsets"][0]) == ["1.2.3.4"]
    assert ep["subsets"][0]["ports"][0]["port"] == 9376


@pytest.mark.parametrize("restart,phase,listed", [("Never", "Failed", False), ("Never", "Succeeded", False),
                                                  ("OnFailure", "Succeeded", False), ("OnFailure", "Failed", True),
                                                  ("Always", "Failed", True)])
def test_not_ready_pods_by_restart_policy(restart, phase, listed):
    ep, _ = sync(svc({"foo": "bar"}), *pods(1, ready=False, restart=restart, phase=phase))
    got = [a["ip"] for ss in ep["subsets"] for a in ss.get("notReadyAddresses") or ()]
    assert got == (["1.2.3.4"] if listed else [])


def test_should_pod_be_in_endpoints():
    assert should_pod_be_in_endpoints({"spec": {"restartPolicy": "Never"}, "status": {"phase": "Running"}})
    assert not should_pod_be_in_endpoints({"spec": {"restartPolicy": "Never"}, "status": {"phase": "Succeeded"}})
    assert should_pod_be_in_endpoints({"spec": {}, "status": {"phase": "Succeeded"}})


@pytest.mark.parametrize("how", ["annotation", "publishNotReadyAddresses"])
def test_tolerate_unready_lists_everything_ready(how):
    s = svc({"foo": "bar"}, publishNotReadyAddresses=True) if how != "annotation" else svc({"foo": "bar"})
    if how == "annotation":
        s["metadata"]["annotations"] = {"service.alpha.kubernetes.io/tolerate-unready-endpoints": "true"}
    dying = pods(1, start=2)[0]
    dying["metadata"]["deletionTimestamp"] = "2017-01-01T00:00:00Z"
    ep, _ = sync(s, *pods(1), *pods(1, ready=False, start=1), dying)
    assert ips(ep["subsets"][0]) == ["1.2.3.4", "1.2.3.5", "1.2.3.6"]
    assert not ep["subsets"][0].get("notReadyAddresses")


def test_terminating_pod_dropped_without_tolerance():
    dying = pods(1)[0]
    dying["metadata"]["deletionTimestamp"] = "2017-01-01T00:00:00Z"
    ep, _ = sync(svc({"foo": "bar"}), dying)
    assert ep["subsets"] == []


def test_headless_service_without_ports():
    ep0 = {"apiVersion": "v1", "kind": "Endpoints", "metadata": {"name": "foo", "namespace": NS, "resourceVersion": "1"},
           "subsets": [{"addresses": [{"ip": "6.7.8.9"}], "ports": [{"port": 1000, "protocol": "TCP"}]}]}
    ep, writes = sync(svc({}, [], clusterIP="None"), ep0, *pods(1, ports=1))
    assert [w.verb for w in writes] == ["update"]
    assert ep["subsets"] == [{"addresses": [ep["subsets"][0]["addresses"][0]], "ports": [{"port": 0, "protocol": "TCP"}]}]
    assert ips(ep["subsets"][0]) == ["1.2.3.4"]


def test_hostname_published_for_matching_subdomain():
    p = pods(2)
    for x in p:
        x["spec"]["hostname"] = x["metadata"]["name"]
    p[0]["spec"]["subdomain"] = "foo"
    p[1]["spec"]["subdomain"] = "other"
    ep, _ = sync(svc({"foo": "bar"}), *p)
    hn = {a["ip"]: a.get("hostname") for a in ep["subsets"][0]["addresses"]}
    assert hn == {"1.2.3.4": "pod0", "1.2.3.5": None}


def test_labels_propagate_and_identical_endpoints_are_not_rewritten():
    s = svc({"foo": "bar"})
    s["metadata"]["labels"] = {"foo": "bar", "baz": "blah"}
    ep, writes = sync(s, *pods(1))
    assert ep["metadata"]["labels"] == {"foo": "bar", "baz": "blah"}
    ep2, writes2 = sync(s, *pods(1), ep)       # same insertion order: same fake resourceVersions
    assert not writes2
    s["metadata"]["labels"] = {"foo": "bar", "baz": "changed"}
    ep3, writes3 = sync(s, *pods(1), ep)
    assert [w.verb for w in writes3] == ["update"] and ep3["metadata"]["labels"]["baz"] == "changed"


def test_deleted_service_deletes_its_endpoints():
    ep0 = {"apiVersion": "v1", "kind": "Endpoints", "metadata": {"name": "foo", "namespace": NS}, "subsets": []}
    ep, writes = sync(ep0)
    assert [w.verb for w in writes] == ["delete"] and ep is None


def test_leftover_endpoints_are_queued_at_start():
    async def main():
        ep0 = {"apiVersion": "v1", "kind": "Endpoints", "metadata": {"name": "foo", "namespace": NS}, "subsets": []}
        leader = {"apiVersion": "v1", "kind": "Endpoints",
                  "metadata": {"name": "kube-scheduler", "namespace": "kube-system",
                               "annotations": {"control-plane.alpha.kubernetes.io/leader": "{}"}}}
        c = FakeClient(ep0, leader)
        f = InformerFactory(c)
        ec = EndpointsController(c, f)
        ec.setup()
        f.start()
        await f.wait_for_cache_sync()
        ec.start()
        for _ in range(100):
            if (NS, "foo") not in c.objects.get("endpoints", {}):
                break
            await asyncio.sleep(0.01)
        ec.stop()
        return c.objects.get("endpoints", {})
    left = asyncio.run(main())
    assert (NS, "foo") not in left and ("kube-system", "kube-scheduler") in left


def test_repack_merges_ports_with_the_same_addresses():
    a = {"ip": "1.1.1.1", "targetRef": {"uid": "a"}}
    b = {"ip": "2.2.2.2", "targetRef": {"uid": "b"}}
    out = repack_subsets([(a, {"name": "p", "port": 1}, True), (b, {"name": "p", "port": 1}, True),
                          (a, {"name": "q", "port": 2}, True), (b, {"name": "q", "port": 2}, False)])
    assert len(out) == 2
    both = [ss for ss in out if len(ss.get("addresses") or ()) == 2][0]
    assert [p["name"] for p in both["ports"]] == ["p"]
    split = [ss for ss in out if ss.get("notReadyAddresses")][0]
    assert ips(split) == ["1.1.1.1"] and ips(split, "notReadyAddresses") == ["2.2.2.2"]
