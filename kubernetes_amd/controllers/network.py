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

import ipaddress

from ..client.rest import APIStatusError, is_not_found
from .base import Controller, split_key


class CIDRSet:
    def __init__(self, cluster_cidr, mask):
        self.net = ipaddress.ip_network(cluster_cidr, strict=False)
        if mask < self.net.prefixlen:
            raise ValueError(f"node CIDR mask /{mask} is larger than the cluster CIDR {cluster_cidr}")
        self.mask = mask
        self.max = 1 << (mask - self.net.prefixlen)
        self.used: set[int] = set()
        self.next = 0

    def _index(self, cidr):
        sub = ipaddress.ip_network(cidr, strict=False)
        if sub.prefixlen != self.mask or not sub.subnet_of(self.net):
            return None
        return (int(sub.network_address) - int(self.net.network_address)) >> (sub.max_prefixlen - self.mask)

    def _cidr(self, i):
        base = int(self.net.network_address) + (i << (self.net.max_prefixlen - self.mask))
        return str(ipaddress.ip_network((base, self.mask)))

    def occupy(self, cidr):
        i = self._index(cidr)
        if i is None:
            return False
        self.used.add(i)
        return True

    def release(self, cidr):
        i = self._index(cidr)
        if i is not None:
            self.used.discard(i)

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

    def __init__(self, client, factory, cluster_cidr="10.244.0.0/16", node_cidr_mask_size=24, **kw):
        super().__init__(client, factory, **kw)
        self.cidrs = CIDRSet(cluster_cidr, node_cidr_mask_size)
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
        cidr = self.owner.get(key) or self.cidrs.allocate()
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
