"""Service / endpoints state for the proxiers.

Parity: `pkg/proxy/service.go` (`ServicePortName` = namespace/name:port-name, per-port
`serviceInfo`: clusterIP, port, protocol, nodePort, externalIPs, loadBalancer ingress,
sessionAffinity + timeout (default 10800 s), `onlyNodeLocalEndpoints` for
`externalTrafficPolicy: Local`, healthCheckNodePort) and `pkg/proxy/endpoints.go`
(per service port: the ready endpoint `ip:port` list with `isLocal` = on this node), plus
`pkg/proxy/config/config.go` (informer handlers feeding a change tracker; the proxier syncs on
changes, rate-limited by `--iptables-min-sync-period`).
"""
from __future__ import annotations

from dataclasses import dataclass, field

DEFAULT_AFFINITY_TIMEOUT = 10800


@dataclass(frozen=True)
class ServicePortName:
    namespace: str
    name: str
    port: str       # port name ("" for a single unnamed port)

    def __str__(self):
        return f"{self.namespace}/{self.name}" + (f":{self.port}" if self.port else "")


@dataclass
class ServiceInfo:
    cluster_ip: str
    port: int
    protocol: str
    node_port: int = 0
    target_port: object = None
    external_ips: list = field(default_factory=list)
    load_balancer_ips: list = field(default_factory=list)
    load_balancer_source_ranges: list = field(default_factory=list)
    session_affinity: str = "None"
    sticky_seconds: int = DEFAULT_AFFINITY_TIMEOUT
    only_local: bool = False
    health_check_node_port: int = 0


@dataclass(frozen=True)
class Endpoint:
    ip: str
    port: int
    is_local: bool = False

    @property
    def endpoint(self):
        return f"{self.ip}:{self.port}"


def services_from(svc) -> dict:
    """Service object -> {ServicePortName: ServiceInfo} (headless / ExternalName skipped)."""
    sp = svc.get("spec") or {}
    md = svc.get("metadata") or {}
    ip = sp.get("clusterIP")
    if not ip or ip == "None" or sp.get("type") == "ExternalName":
        return {}
    out = {}
    aff = sp.get("sessionAffinity", "None")
    timeout = ((sp.get("sessionAffinityConfig") or {}).get("clientIP") or {}).get("timeoutSeconds") or DEFAULT_AFFINITY_TIMEOUT
    lbs = [i.get("ip") for i in ((svc.get("status") or {}).get("loadBalancer") or {}).get("ingress") or () if i.get("ip")]
    only_local = sp.get("externalTrafficPolicy") == "Local" and sp.get("type") in ("NodePort", "LoadBalancer")
    for p in sp.get("ports") or ():
        name = ServicePortName(md.get("namespace", ""), md.get("name", ""), p.get("name", ""))
        out[name] = ServiceInfo(ip, int(p["port"]), p.get("protocol", "TCP"), int(p.get("nodePort") or 0),
                                p.get("targetPort", p["port"]), list(sp.get("externalIPs") or []), lbs,
                                list(sp.get("loadBalancerSourceRanges") or []), aff, int(timeout), only_local,
                                int(sp.get("healthCheckNodePort") or 0))
    return out


def endpoints_from(ep, hostname) -> dict:
    """Endpoints object -> {ServicePortName: [Endpoint]} (ready addresses only)."""
    md = ep.get("metadata") or {}
    out: dict = {}
    for ss in ep.get("subsets") or ():
        for port in ss.get("ports") or ():
            name = ServicePortName(md.get("namespace", ""), md.get("name", ""), port.get("name", ""))
            lst = out.setdefault(name, [])
            for a in ss.get("addresses") or ():
                e = Endpoint(a["ip"], int(port["port"]), a.get("nodeName") == hostname)
                if e not in lst:
                    lst.append(e)
    for lst in out.values():
        lst.sort(key=lambda e: (e.ip, e.port))
    return out


class ProxyState:
    """Current service and endpoints maps plus a dirty flag (the change trackers)."""

    def __init__(self, hostname):
        self.hostname = hostname
        self.services: dict = {}           # ServicePortName -> ServiceInfo
        self.endpoints: dict = {}          # ServicePortName -> [Endpoint]
        self._svc_by_obj: dict = {}        # ns/name -> set(ServicePortName)
        self._ep_by_obj: dict = {}
        self.listeners = []

    def _changed(self):
        for fn in self.listeners:
            fn()

    def on_service(self, svc, deleted=False):
        key = f"{svc['metadata'].get('namespace', '')}/{svc['metadata']['name']}"
        for n in self._svc_by_obj.pop(key, ()):
            self.services.pop(n, None)
        if not deleted:
            m = services_from(svc)
            self.services.update(m)
            self._svc_by_obj[key] = set(m)
        self._changed()

    def on_endpoints(self, ep, deleted=False):
        key = f"{ep['metadata'].get('namespace', '')}/{ep['metadata']['name']}"
        for n in self._ep_by_obj.pop(key, ()):
            self.endpoints.pop(n, None)
        if not deleted:
            m = endpoints_from(ep, self.hostname)
            self.endpoints.update(m)
            self._ep_by_obj[key] = set(m)
        self._changed()

    def attach(self, svc_informer, ep_informer):
        svc_informer.add_handler(self.on_service, lambda o, n: self.on_service(n), lambda s: self.on_service(s, True))
        ep_informer.add_handler(self.on_endpoints, lambda o, n: self.on_endpoints(n), lambda e: self.on_endpoints(e, True))
