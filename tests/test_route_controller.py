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


def test_ip_routes_lists_kernel_table():
    """`list()` reads the kernel table: gateways map back to nodes, blackhole and
    unreachable entries are blackholes, connected routes are not node routes."""
    out = ("10.244.1.0/24 via 10.0.0.11 dev eth0 \n"
           "10.244.2.0/24 via 10.0.0.99 dev eth0 proto static\n"
           "blackhole 10.244.7.0/24 \n"
           "unreachable 10.244.8.0/24 \n"
           "10.244.0.0/24 dev cni0 proto kernel scope link src 10.244.0.1\n")
    calls = []

    def runner(argv):
        calls.append(argv)
        return out if argv[:3] == ["ip", "-o", "route"] else None
    t = IPRoutes({"gpu-1": "10.0.0.11"}.get, runner=runner, cluster_cidr="10.244.0.0/16",
                 node_by_ip={"10.0.0.11": "gpu-1"}.get)
    rs = {r["destinationCIDR"]: r for r in t.list()}
    assert calls[0] == ["ip", "-o", "route", "show", "root", "10.244.0.0/16"]
    assert rs["10.244.1.0/24"]["targetNode"] == "gpu-1" and not rs["10.244.1.0/24"]["blackhole"]
    assert rs["10.244.2.0/24"]["targetNode"] == ""          # gateway of no known node: stale
    assert rs["10.244.7.0/24"]["blackhole"] and rs["10.244.8.0/24"]["blackhole"]
    assert "10.244.0.0/24" not in rs
    t.delete(rs["10.244.8.0/24"])
    assert calls[-1] == ["ip", "route", "del", "unreachable", "10.244.8.0/24"]


def test_route_follows_pod_cidr_change_and_periodic_reconcile(run):
    """A node re-created with another podCIDR keeps one route (the re-created route under the same name
    hint is not deleted as stale), and a route removed outside the controller comes back on the
    periodic reconcile without any node event."""
    table = MemoryRoutes()

    async def main():
        s = APIServer()
        c = Client(f"http://127.0.0.1:{await s.start()}")
        await c.create("nodes", {"metadata": {"name": "n1"}, "spec": {"podCIDR": "10.244.1.0/24"}, "status": {}})
        cm = await ControllerManager(c, ["route"], {"route": {"cluster_cidr": "10.244.0.0/16", "routes": table,
                                                              "reconcile_period": 0.2}}).start()
        try:
            async def dests():
                for _ in range(200):
                    await asyncio.sleep(0.02)
                    yield sorted(r["destinationCIDR"] for r in table.list())
            async for d in dests():
                if d == ["10.244.1.0/24"]:
                    break
            # podCIDR is set-once (ValidateNodeUpdate): the node is re-created with another one
            await c.delete("nodes", "n1")
            await c.create("nodes", {"metadata": {"name": "n1"}, "spec": {"podCIDR": "10.244.5.0/24"}, "status": {}})
            async for d in dests():
                if d == ["10.244.5.0/24"]:
                    break
            await asyncio.sleep(0.3)
            assert sorted(r["destinationCIDR"] for r in table.list()) == ["10.244.5.0/24"]
            table.routes.clear()                     # deleted behind the controller's back
            async for d in dests():
                if d == ["10.244.5.0/24"]:
                    break
            assert sorted(r["destinationCIDR"] for r in table.list()) == ["10.244.5.0/24"]
        finally:
            await cm.stop()
            await c.close()
            await s.stop()
    run(main())
