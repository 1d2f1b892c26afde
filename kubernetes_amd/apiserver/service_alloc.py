"""Service ClusterIP / NodePort allocation and Service validation.

Parity: `pkg/registry/core/service/storage/rest.go` (Create: allocate `spec.clusterIP` from
`--service-cluster-ip-range` unless `None` (headless) or ExternalName, allocate a NodePort per
port for NodePort/LoadBalancer services from `--service-node-port-range` 30000-32767, release on
delete, keep them across updates), `pkg/registry/core/service/ipallocator` /
`portallocator` (bitmap allocators persisted in etcd as RangeAllocation objects) and
`pkg/apis/core/validation/validation.go` ValidateService.

Uniqueness: within one API server the watch cache is authoritative; across API server workers
sharing the native store every allocated IP / port is also a claim key written in the same
transaction as the Service (`CMP_ABSENT`), like the GPU device claims — the store rejects a
double allocation atomically.
"""
from __future__ import annotations

import ipaddress
import random

from ..api import validation as v

IP_PREFIX = "/kamd/ranges/serviceips/"
PORT_PREFIX = "/kamd/ranges/servicenodeports/"
TYPES = ("ClusterIP", "NodePort", "LoadBalancer", "ExternalName")


class AllocationError(Exception):
    def __init__(self, code, msg):
        super().__init__(msg)
        self.code = code


class ServiceAllocator:
    def __init__(self, cidr="10.0.0.0/24", node_ports=(30000, 32767)):
        self.net = ipaddress.ip_network(cidr)
        self.node_ports = node_ports
        # network and broadcast addresses are never allocated; the first usable IP is reserved
        # for the `kubernetes` service (master.go: DefaultServiceIPRange -> .1)
        self.first = int(self.net.network_address) + 1
        self.last = int(self.net.broadcast_address) - 1

    @property
    def kubernetes_ip(self):
        return str(ipaddress.ip_address(self.first))

    def contains(self, ip):
        try:
            a = ipaddress.ip_address(ip)
        except ValueError:
            return False
        return a in self.net and self.first <= int(a) <= self.last

    def used(self, services):
        ips, ports = set(), set()
        for s in services:
            sp = s.get("spec") or {}
            ip = sp.get("clusterIP")
            if ip and ip != "None":
                ips.add(ip)
            for p in sp.get("ports") or ():
                if p.get("nodePort"):
                    ports.add((p.get("protocol", "TCP"), int(p["nodePort"])))
        return ips, ports

    def allocate(self, svc, services, rng=random):
        """Fill in clusterIP / nodePorts of a new Service. Returns True if anything was
        auto-allocated (the caller may retry on a cross-worker claim conflict)."""
        sp = svc.setdefault("spec", {})
        typ = sp.setdefault("type", "ClusterIP")
        if typ == "ExternalName":
            sp.pop("clusterIP", None)
            return False
        sp.setdefault("sessionAffinity", "None")
        ips, ports = self.used(services)
        auto = False
        ip = sp.get("clusterIP")
        if ip == "None":
            pass
        elif ip:
            if not self.contains(ip):
                raise AllocationError(422, f'spec.clusterIP: Invalid value: "{ip}": provided IP is not in the valid range. '
                                           f"The range of valid IPs is {self.net}")
            if ip in ips:
                raise AllocationError(422, f'spec.clusterIP: Invalid value: "{ip}": provided IP is already allocated')
        else:
            free = self.last - self.first + 1 - len(ips)
            if free <= 0:
                raise AllocationError(500, "Internal error occurred: failed to allocate a serviceIP: range is full")
            for _ in range(64):
                cand = str(ipaddress.ip_address(rng.randint(self.first + 1, self.last)))
                if cand not in ips:
                    break
            else:
                cand = next(str(ipaddress.ip_address(i)) for i in range(self.first + 1, self.last + 1)
                            if str(ipaddress.ip_address(i)) not in ips)
            sp["clusterIP"] = cand
            auto = True
        if typ in ("NodePort", "LoadBalancer"):
            lo, hi = self.node_ports
            for p in sp.get("ports") or ():
                proto = p.get("protocol", "TCP")
                np = p.get("nodePort")
                if np:
                    np = int(np)
                    if not lo <= np <= hi:
                        raise AllocationError(422, f"spec.ports.nodePort: Invalid value: {np}: provided port is not in the valid range. "
                                                   f"The range of valid ports is {lo}-{hi}")
                    if (proto, np) in ports:
                        raise AllocationError(422, f"spec.ports.nodePort: Invalid value: {np}: provided port is already allocated")
                else:
                    for _ in range(256):
                        np = rng.randint(lo, hi)
                        if (proto, np) not in ports:
                            break
                    p["nodePort"] = np
                    auto = True
                ports.add((proto, np))
        else:
            for p in sp.get("ports") or ():
                p.pop("nodePort", None)
        return auto

    @staticmethod
    def claim_keys(svc):
        if svc is None:
            return set()
        sp = svc.get("spec") or {}
        keys = set()
        ip = sp.get("clusterIP")
        if ip and ip != "None":
            keys.add(IP_PREFIX + ip)
        for p in sp.get("ports") or ():
            if p.get("nodePort"):
                keys.add(f"{PORT_PREFIX}{p.get('protocol', 'TCP')}/{int(p['nodePort'])}")
        return keys


def validate_service(svc):
    errs = v.validate_object_meta(svc, True, v.is_dns1123_label)
    sp = svc.get("spec") or {}
    typ = sp.get("type", "ClusterIP")
    if typ not in TYPES:
        errs.append(v.not_supported("spec.type", typ))
    if typ == "ExternalName":
        if not sp.get("externalName"):
            errs.append(v.required("spec.externalName"))
        return errs
    ports = sp.get("ports") or []
    if not ports and sp.get("clusterIP") != "None":
        errs.append(v.required("spec.ports"))
    names = set()
    for i, p in enumerate(ports):
        path = f"spec.ports[{i}]"
        port = p.get("port")
        if not isinstance(port, int) or not 1 <= port <= 65535:
            errs.append(v.invalid(f"{path}.port", "must be between 1 and 65535, inclusive"))
        if p.get("protocol", "TCP") not in ("TCP", "UDP"):
            errs.append(v.not_supported(f"{path}.protocol", p.get("protocol")))
        if len(ports) > 1 and not p.get("name"):
            errs.append(v.required(f"{path}.name", "must be specified when there is more than one port"))
        if p.get("name"):
            if p["name"] in names:
                errs.append(v.duplicate(f"{path}.name", p["name"]))
            names.add(p["name"])
        tp = p.get("targetPort")
        if isinstance(tp, int) and not 1 <= tp <= 65535:
            errs.append(v.invalid(f"{path}.targetPort", "must be between 1 and 65535, inclusive"))
    if sp.get("sessionAffinity", "None") not in ("None", "ClientIP"):
        errs.append(v.not_supported("spec.sessionAffinity", sp.get("sessionAffinity")))
    if sp.get("externalTrafficPolicy") and sp["externalTrafficPolicy"] not in ("Cluster", "Local"):
        errs.append(v.not_supported("spec.externalTrafficPolicy", sp["externalTrafficPolicy"]))
    if sp.get("externalTrafficPolicy") == "Local" and typ not in ("NodePort", "LoadBalancer"):
        errs.append(v.invalid("spec.externalTrafficPolicy", "may only be set when `type` is 'NodePort' or 'LoadBalancer'"))
    return errs


def validate_service_update(new, old):
    errs = validate_service(new)
    ns, os_ = new.get("spec") or {}, old.get("spec") or {}
    if os_.get("clusterIP") and os_.get("clusterIP") != ns.get("clusterIP") and os_.get("type") != "ExternalName" \
            and ns.get("type") != "ExternalName":
        errs.append(v.invalid("spec.clusterIP", "field is immutable"))
    return errs
