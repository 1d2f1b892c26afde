"""Network controllers: node IPAM (pod CIDR range allocator) and the LoadBalancer service
controller.

Parity:
  * NodeIPAM — `pkg/controller/node/ipam/range_allocator.go` (`--allocate-node-cidrs`,
    `--cluster-cidr`, `--node-cidr-mask-size` 24): on start every existing `spec.podCIDR` is
    marked used; a node without one gets the next free subnet (`cidrset.go` round-robin from
    the last allocation); a deleted node's subnet is released. A node whose recorded CIDR
    lies outside the cluster CIDR is left alone (the reference logs and skips it).
  * Service — `pkg/controller/service/service_controller.go` drives a cloud load balancer
    for `type: LoadBalancer` services. On an MI355X on-prem node there is no cloud, so the
    controller assigns ingress IPs from a configured pool (`--loadbalancer-ip-range`; honours
    `spec.loadBalancerIP` when it is in the pool and free) into `status.loadBalancer.ingress`,
    and releases them when the service is deleted or changes type. kube-proxy already
    forwards traffic for ingress IPs (`proxy/iptables.py` KUBE-FW chains).
"""
from __future__ import annotations

import asyncio
import ipaddress

from ..api.meta import now_rfc3339
from ..client.rest import APIStatusError, is_not_found
from .base import Controller, split_key


CLUSTER_SUBNET_MAX_DIFF = 16      # `cidrset.clusterSubnetMaxDiff` (IPv6 only)


class CIDRSet:
    """`pkg/controller/node/ipam/cidrset/cidr_set.go`: the cluster CIDR cut into /mask node
    blocks, allocated round-robin from the last allocation; Occupy / Release take any CIDR and
    mark every block it overlaps (`getBeginingAndEndIndices`), refusing one outside the
    cluster range."""

    def __init__(self, cluster_cidr, mask):
        self.net = ipaddress.ip_network(cluster_cidr, strict=False)
        if mask < self.net.prefixlen:
            raise ValueError(f"node CIDR mask /{mask} is larger than the cluster CIDR {cluster_cidr}")
        if self.net.version == 6 and mask - self.net.prefixlen > CLUSTER_SUBNET_MAX_DIFF:
            raise ValueError("New CIDR set failed; the node CIDR size is too big")
        self.mask = mask
        self.max = 1 << (mask - self.net.prefixlen)
        self.used: set[int] = set()
        self.next = 0
        self._net_cls = ipaddress.IPv4Network if self.net.version == 4 else ipaddress.IPv6Network

    def _indices(self, cidr):
        """(first, last) block indices `cidr` overlaps, or None when it is outside the cluster
        range (neither contains the other's base address)."""
        other = ipaddress.ip_network(cidr, strict=False)
        if other.version != self.net.version or not (other.network_address in self.net or
                                                     self.net.network_address in other):
            return None
        lo = max(int(self.net.network_address), int(other.network_address))
        hi = min(int(self.net.broadcast_address), int(other.broadcast_address))
        shift = self.net.max_prefixlen - self.mask
        return (lo - int(self.net.network_address)) >> shift, (hi - int(self.net.network_address)) >> shift

    def _cidr(self, i):
        base = int(self.net.network_address) + (i << (self.net.max_prefixlen - self.mask))
        return str(self._net_cls((base, self.mask)))

    def occupy(self, cidr):
        r = self._indices(cidr)
        if r is None:
            return False
        self.used.update(range(r[0], r[1] + 1))
        return True

    def exclude(self, cidr):
        """Mark every node block that overlaps `cidr` used (`filterOutServiceRange` of
        pkg/controller/node/ipam/range_allocator.go: the service range is never a pod CIDR)."""
        other = ipaddress.ip_network(cidr, strict=False)
        if other.version != self.net.version or not self.net.overlaps(other):
            return 0
        first, last = self._indices(cidr)
        self.used.update(range(first, last + 1))
        return last - first + 1

    def release(self, cidr):
        r = self._indices(cidr)
        if r is not None:
            self.used.difference_update(range(r[0], r[1] + 1))

    def allocate(self):
        for k in range(self.max):
            i = (self.next + k) % self.max
            if i not in self.used:
                self.used.add(i)
                self.next = (i + 1) % self.max
                return self._cidr(i)
        raise RuntimeError("CIDR allocation failed; there are no remaining CIDRs left to allocate in the accepted range")


class NodeIPAMController(Controller):
    name = "nodeipam"
    workers = 1

    def __init__(self, client, factory, cluster_cidr="10.244.0.0/16", node_cidr_mask_size=24,
                 service_cluster_ip_range="", **kw):
        super().__init__(client, factory, **kw)
        self.cidrs = CIDRSet(cluster_cidr, node_cidr_mask_size)
        if service_cluster_ip_range:          # --service-cluster-ip-range
            self.cidrs.exclude(service_cluster_ip_range)
        self.owner: dict[str, str] = {}          # node name -> allocated CIDR

    def setup(self):
        self.node_inf = self.factory.get("nodes")
        self.node_inf.add_handler(self._add, lambda o, n: self._add(n), self._delete)

    def _add(self, node):
        cidr = (node.get("spec") or {}).get("podCIDR")
        name = node["metadata"]["name"]
        if cidr:
            if self.owner.get(name) != cidr and self.cidrs.occupy(cidr):
                self.owner[name] = cidr
            return
        self.enqueue(name)

    def _delete(self, node):
        name = node["metadata"]["name"]
        cidr = self.owner.pop(name, None) or (node.get("spec") or {}).get("podCIDR")
        if cidr:
            self.cidrs.release(cidr)

    async def sync(self, key):
        node = self.node_inf.get(key)
        if node is None or (node.get("spec") or {}).get("podCIDR"):
            return
        try:
            cidr = self.owner.get(key) or self.cidrs.allocate()
        except RuntimeError:
            # `AllocateOrOccupyCIDR`: recordNodeStatusChange(CIDRNotAvailable), then retried
            self.recorder.event(node, "Normal", "CIDRNotAvailable", f"Node {key} status is now: CIDRNotAvailable")
            raise
        self.owner[key] = cidr
        try:
            await self.client.patch("nodes", key, {"spec": {"podCIDR": cidr}})
        except APIStatusError as e:
            if is_not_found(e):
                self.cidrs.release(cidr)
                self.owner.pop(key, None)
                return
            raise


def _range(spec):
    """'10.0.5.10-10.0.5.50' or a CIDR."""
    if not spec:
        return []
    if "-" in spec:
        lo, hi = (ipaddress.ip_address(x.strip()) for x in spec.split("-", 1))
        return [str(ipaddress.ip_address(i)) for i in range(int(lo), int(hi) + 1)]
    return [str(h) for h in ipaddress.ip_network(spec, strict=False).hosts()]


class ServiceLBController(Controller):
    name = "service"
    primary = "services"
    workers = 1

    def __init__(self, client, factory, ip_range="", **kw):
        super().__init__(client, factory, **kw)
        self.pool = _range(ip_range)
        self.assigned: dict[str, str] = {}       # ns/name -> ip

    def setup(self):
        self.svc_inf = self.factory.get("services")
        self.svc_inf.add_handler(self._event, lambda o, n: self._event(n), self._gone)

    def _event(self, svc):
        md = svc["metadata"]
        key = f"{md['namespace']}/{md['name']}"
        for ing in ((svc.get("status") or {}).get("loadBalancer") or {}).get("ingress") or ():
            if ing.get("ip") in self.pool and key not in self.assigned:
                self.assigned[key] = ing["ip"]
        self.enqueue(key)

    def _gone(self, svc):
        md = svc["metadata"]
        if self.assigned.pop(f"{md['namespace']}/{md['name']}", None):
            self._requeue_waiting()

    def _requeue_waiting(self):
        """An address went back to the pool: retry services still waiting for one."""
        for s in self.svc_inf.list():
            md = s["metadata"]
            k = f"{md['namespace']}/{md['name']}"
            if (s.get("spec") or {}).get("type") == "LoadBalancer" and k not in self.assigned:
                self.enqueue(k)

    def _pick(self, want):
        used = set(self.assigned.values())
        if want:
            return want if want in self.pool and want not in used else None
        return next((ip for ip in self.pool if ip not in used), None)

    async def sync(self, key):
        svc = self.svc_inf.get(key)
        if svc is None:
            if self.assigned.pop(key, None):
                self._requeue_waiting()
            return
        ns, name = split_key(key)
        spec = svc.get("spec") or {}
        cur = ((svc.get("status") or {}).get("loadBalancer") or {}).get("ingress") or []
        if spec.get("type") != "LoadBalancer":
            if key in self.assigned or cur:
                freed = self.assigned.pop(key, None)
                await self.client.patch("services", name, {"status": {"loadBalancer": {"ingress": None}}}, ns, "merge", "status")
                if freed:
                    self._requeue_waiting()
            return
        ip = self.assigned.get(key)
        if ip is None:
            ip = self._pick(spec.get("loadBalancerIP"))
            if ip is None:
                self.recorder.event(svc, "Warning", "CreatingLoadBalancerFailed",
                                    f"no free address in the load-balancer pool for {spec.get('loadBalancerIP') or key}")
                return
            self.assigned[key] = ip
        if cur != [{"ip": ip}]:
            await self.client.patch("services", name, {"status": {"loadBalancer": {"ingress": [{"ip": ip}]}}}, ns,
                                    "merge", "status")


class MemoryRoutes:
    """Route table behind the route controller (the reference's `cloudprovider.Routes`):
    `list()` → [{"name", "targetNode", "destinationCIDR", "blackhole"}], `create(hint, route)`,
    `delete(route)`. This one keeps the table in memory (tests, single-host clusters)."""

    def __init__(self, routes=None):
        self.routes: dict[str, dict] = {r["name"]: dict(r) for r in routes or ()}
        self.fail: set[str] = set()          # target nodes whose creation fails (fault injection)

    def list(self):
        return [dict(r) for r in self.routes.values()]

    def create(self, hint, route):
        if route["targetNode"] in self.fail:
            raise RuntimeError(f"route to {route['targetNode']} refused")
        self.routes[hint] = dict(route, name=hint, blackhole=False)

    def delete(self, route):
        # a route is identified by name AND destination: a stale listing can name a route that
        # has since been re-created under the same hint for a new CIDR
        cur = self.routes.get(route["name"])
        if cur is not None and cur["destinationCIDR"] == route["destinationCIDR"]:
            del self.routes[route["name"]]


class IPRoutes(MemoryRoutes):
    """On-prem route table on a gateway host: `ip route replace <podCIDR> via <node InternalIP>`
    (`ip route del` on removal). `list()` reads the kernel table (`ip -o route show root
    <clusterCIDR>`), mapping each gateway back to its node through the nodes' InternalIPs and
    reporting `blackhole`/`unreachable`/`prohibit` entries as blackholes, so routes deleted or
    added behind the controller's back — or left over from before a restart — are reconciled.
    Connected (`dev`-only) routes, e.g. the gateway's own bridge, are never reported.
    `runner` executes argv lists and returns their stdout (str/bytes/CompletedProcess); a
    runner that returns nothing (dry-run) falls back to the in-memory view."""

    BLACKHOLE_TYPES = ("blackhole", "unreachable", "prohibit")

    def __init__(self, node_ip, runner=None, cluster_cidr="0.0.0.0/0", node_by_ip=None):
        super().__init__()
        self.node_ip = node_ip               # node name -> InternalIP
        self.node_by_ip = node_by_ip or (lambda ip: None)
        self.cluster_cidr = cluster_cidr
        import subprocess
        self.runner = runner or (lambda argv: subprocess.run(argv, check=True, capture_output=True, text=True).stdout)

    @staticmethod
    def _text(out):
        if out is None:
            return None
        out = getattr(out, "stdout", out)
        return out.decode() if isinstance(out, (bytes, bytearray)) else out

    def parse(self, text):
        routes = []
        for ln in text.splitlines():
            f = ln.split()
            if not f:
                continue
            kind = "unicast"
            if f[0] in self.BLACKHOLE_TYPES + ("unicast", "local", "broadcast", "multicast", "throw", "nat"):
                kind, f = f[0], f[1:]
            if not f or kind not in ("unicast",) + self.BLACKHOLE_TYPES:
                continue
            dst = f[0]
            if "/" not in dst:
                dst += "/32"
            if kind in self.BLACKHOLE_TYPES:
                routes.append({"name": f"{kind}:{dst}", "targetNode": "", "destinationCIDR": dst, "blackhole": True,
                               "type": kind})
                continue
            if "via" not in f:
                continue                      # connected route: not a node route
            gw = f[f.index("via") + 1]
            node = self.node_by_ip(gw) or ""
            routes.append({"name": f"{node or gw}:{dst}", "targetNode": node, "destinationCIDR": dst,
                           "blackhole": False, "via": gw})
        return routes

    def list(self):
        text = self._text(self.runner(["ip", "-o", "route", "show", "root", self.cluster_cidr]))
        if text is None:
            return super().list()
        return self.parse(text)

    def create(self, hint, route):
        ip = self.node_ip(route["targetNode"])
        if not ip:
            raise RuntimeError(f"node {route['targetNode']} has no InternalIP")
        self.runner(["ip", "route", "replace", route["destinationCIDR"], "via", ip])
        super().create(hint, route)

    def delete(self, route):
        argv = ["ip", "route", "del"]
        if route.get("blackhole"):
            argv.append(route.get("type") or "blackhole")
        self.runner(argv + [route["destinationCIDR"]])
        super().delete(route)


class RouteController(Controller):
    """`pkg/controller/route/route_controller.go:123-262`: every node with a `spec.podCIDR`
    gets a route to it (created with the node UID as name hint, up to `MAX_RETRIES` tries,
    `FailedToCreateRoute` event on failure); the node's `NetworkUnavailable` condition is set
    False/`RouteCreated` once its route exists and True/`NoRouteCreated` when creation failed;
    routes inside the cluster CIDR that are blackholes or point at a node with a different (or
    no) CIDR are deleted. On-prem there is no cloud route API, so the table is pluggable
    (`MemoryRoutes`, `IPRoutes`). All nodes reconcile under one key, as the reference's
    periodic `reconcileNodeRoutes`."""
    name = "route"
    workers = 1
    MAX_RETRIES = 5
    KEY = "routes"

    def __init__(self, client, factory, cluster_cidr="10.244.0.0/16", routes=None, reconcile_period=10.0, **kw):
        super().__init__(client, factory, **kw)
        self.reconcile_period = reconcile_period
        self.cluster = ipaddress.ip_network(cluster_cidr, strict=False)
        if routes == "ip":
            routes = IPRoutes(self._node_ip, cluster_cidr=str(self.cluster), node_by_ip=self._node_by_ip)
        self.routes = routes if routes not in (None, "memory") else MemoryRoutes()

    def _node_ip(self, name):
        node = self.node_inf.get(name) or {}
        return next((a["address"] for a in (node.get("status") or {}).get("addresses") or ()
                     if a.get("type") == "InternalIP"), None)

    def _node_by_ip(self, ip):
        for node in self.node_inf.list():
            if any(a.get("type") == "InternalIP" and a.get("address") == ip
                   for a in (node.get("status") or {}).get("addresses") or ()):
                return node["metadata"]["name"]
        return None

    def setup(self):
        self.node_inf = self.factory.get("nodes")
        self.node_inf.add_handler(lambda n: self.enqueue(self.KEY), lambda o, n: self.enqueue(self.KEY),
                                  lambda n: self.enqueue(self.KEY))

    def start(self):
        """Besides node events, reconcile every `reconcile_period` seconds
        (`route_controller.go` Run: `wait.NonSlidingUntil(reconcileNodeRoutes, syncPeriod)`,
        --route-reconciliation-period, default 10 s): the table can change outside the controller."""
        super().start()

        async def periodic():
            while True:
                await asyncio.sleep(self.reconcile_period)
                self.enqueue(self.KEY)
        self._tasks.append(asyncio.ensure_future(periodic()))

    def _responsible(self, route):
        try:
            return ipaddress.ip_network(route["destinationCIDR"], strict=False).subnet_of(self.cluster)
        except (ValueError, TypeError):
            return False

    async def _set_condition(self, node_name, created):
        now = now_rfc3339()
        cond = ({"type": "NetworkUnavailable", "status": "False", "reason": "RouteCreated",
                 "message": "RouteController created a route"} if created else
                {"type": "NetworkUnavailable", "status": "True", "reason": "NoRouteCreated",
                 "message": "RouteController failed to create a route"})
        cond.update(lastHeartbeatTime=now, lastTransitionTime=now)
        try:
            await self.client.patch("nodes", node_name, {"status": {"conditions": [cond]}}, None, "strategic", "status")
        except APIStatusError as e:
            if not is_not_found(e):
                raise

    async def sync(self, key):
        nodes = self.node_inf.list()
        table = self.routes.list()
        by_target = {r["targetNode"]: r for r in table if r.get("targetNode")}
        cidrs = {}
        for node in nodes:
            name = node["metadata"]["name"]
            cidr = (node.get("spec") or {}).get("podCIDR")
            if not cidr:
                continue
            cidrs[name] = cidr
            r = by_target.get(name)
            if r is None or r["destinationCIDR"] != cidr:
                route = {"targetNode": name, "destinationCIDR": cidr}
                err = None
                for _ in range(self.MAX_RETRIES):
                    try:
                        self.routes.create(node["metadata"].get("uid") or name, route)
                        err = None
                        break
                    except Exception as e:  # noqa: BLE001 - provider errors are retried, then reported
                        err = e
                await self._set_condition(name, err is None)
                if err is not None:
                    self.recorder.event({"kind": "Node", "metadata": {"name": name, "uid": name, "namespace": ""}},
                                        "Warning", "FailedToCreateRoute",
                                        f"Could not create route {cidr} for node {name}: {err}")
            else:
                cur = next((c for c in (node.get("status") or {}).get("conditions") or ()
                            if c.get("type") == "NetworkUnavailable"), None)
                if cur is None or cur.get("status") != "False":
                    await self._set_condition(name, True)
        # re-list: the creates above may have replaced entries of the first listing (a node
        # whose podCIDR changed keeps its name hint), which must not be deleted as stale
        for r in self.routes.list():
            if self._responsible(r) and (r.get("blackhole") or cidrs.get(r.get("targetNode")) != r["destinationCIDR"]):
                self.routes.delete(r)
