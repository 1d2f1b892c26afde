"""Route controller: routes to node pod CIDRs, NetworkUnavailable condition, stale/blackhole
route cleanup, FailedToCreateRoute, and the `ip route` table provider.

Parity: `pkg/controller/route/route_controller_test.go` (reconcile cases: missing route created,
wrong-CIDR route replaced, blackhole deleted, routes outside the cluster CIDR left alone,
NetworkUnavailable updated).
"""
import asyncio

from kubernetes_amd.apiserver.server import APIServer
from kubernetes_amd.client.rest import Client
from kubernetes_amd.controllers.manager import ControllerManager
from kubernetes_amd.controllers.network import IPRoutes, MemoryRoutes


def _cond(node):
    return next((c for c in node["status"].get("conditions") or () if c["type"] == "NetworkUnavailable"), None)


def test_route_controller_reconcile(run):
    table = MemoryRoutes([
        {"name": "stale", "targetNode": "n1", "destinationCIDR": "10.244.9.0/24", "blackhole": False},
        {"name": "hole", "targetNode": "", "destinationCIDR": "10.244.7.0/24", "blackhole": True},
        {"name": "foreign", "targetNode": "", "destinationCIDR": "192.168.5.0/24", "blackhole": True}])
    table.fail.add("n3")

    async def main():
        s = APIServer()
        c = Client(f"http://127.0.0.1:{await s.start()}")
        for name, cidr in (("n1", "10.244.1.0/24"), ("n2", "10.244.2.0/24"), ("n3", "10.244.3.0/24"), ("n4", None)):
            spec = {"podCIDR": cidr} if cidr else {}
            await c.create("nodes", {"metadata": {"name": name}, "spec": spec, "status": {"conditions": [
                {"type": "Ready", "status": "True", "reason": "KubeletReady", "message": ""}]}})
        cm = await ControllerManager(c, ["route"], {"route": {"cluster_cidr": "10.244.0.0/16", "routes": table}}).start()
        try:
            for _ in range(200):
                await asyncio.sleep(0.02)
                n1 = await c.get("nodes", "n1")
                n3 = await c.get("nodes", "n3")
                if _cond(n1) and _cond(n3) and "stale" not in table.routes:
                    break
            dests = sorted((r["targetNode"], r["destinationCIDR"]) for r in table.list())
            assert ("n1", "10.244.1.0/24") in dests and ("n2", "10.244.2.0/24") in dests
            assert not any(r["targetNode"] in ("n3", "n4") for r in table.list())
            assert "stale" not in table.routes and "hole" not in table.routes
            assert "foreign" in table.routes                 # outside the cluster CIDR: not ours
            assert _cond(n1)["status"] == "False" and _cond(n1)["reason"] == "RouteCreated"
            assert any(x["type"] == "Ready" for x in n1["status"]["conditions"])   # strategic merge kept Ready
            assert _cond(n3)["status"] == "True" and _cond(n3)["reason"] == "NoRouteCreated"
            assert any(e[1] == "FailedToCreateRoute" for e in cm.controllers[0].recorder.emitted)
            assert _cond(await c.get("nodes", "n4")) is None
        finally:
            await cm.stop()
            await c.close()
            await s.stop()
    run(main())


def test_ip_routes_provider():
    calls = []
    ips = {"gpu-0": "10.0.0.11"}
    t = IPRoutes(ips.get, runner=calls.append)
    t.create("uid-0", {"targetNode": "gpu-0", "destinationCIDR": "10.244.0.0/24"})
    assert calls == [["ip", "route", "replace", "10.244.0.0/24", "via", "10.0.0.11"]]
    t.delete(t.list()[0])
    assert calls[-1] == ["ip", "route", "del", "10.244.0.0/24"] and t.list() == []
    try:
        t.create("uid-1", {"targetNode": "gpu-9", "destinationCIDR": "10.244.1.0/24"})
    except RuntimeError as e:
        assert "no InternalIP" in str(e)
    else:
        raise AssertionError("expected failure")
