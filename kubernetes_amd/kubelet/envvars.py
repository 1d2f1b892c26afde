"""Service environment variables for containers (`pkg/kubelet/envvars/envvars.go`,
`kubelet_pods.go` getServiceEnvVarMap).

Every container sees, for each service of its namespace plus the `kubernetes` master service of
the master service namespace (`--master-service-namespace`, `default`; headless services, whose ClusterIP is None, are skipped):

    {NAME}_SERVICE_HOST=<clusterIP>          {NAME}_SERVICE_PORT=<first port>
    {NAME}_SERVICE_PORT_{PORTNAME}=<port>    (named ports)
    {NAME}_PORT=tcp://<ip>:<first port>      (Docker-link compatible variables, per port:)
    {NAME}_PORT_<port>_<PROTO>=tcp://<ip>:<port>   …_PROTO / …_PORT / …_ADDR

with NAME the upper-cased service name, '-' → '_'. The container's own `env` wins on a clash
(it is applied after these).
"""
from __future__ import annotations

MASTER_NAMESPACE = "default"
MASTER_SERVICES = ("kubernetes",)


def _upper(s: str) -> str:
    return s.upper().replace("-", "_")


def _ip_set(svc) -> bool:
    ip = (svc.get("spec") or {}).get("clusterIP")
    return bool(ip) and ip != "None"


def service_map(services, namespace, master_namespace=MASTER_NAMESPACE) -> dict:
    """getServiceEnvVarMap: every service of the pod's namespace, plus the master services of
    `--master-service-namespace` unless the pod's namespace has its own of that name."""
    out = {}
    for svc in services:
        if not _ip_set(svc):
            continue
        md = svc["metadata"]
        name, ns = md["name"], md.get("namespace", "default")
        if ns == namespace:
            out[name] = svc
        elif ns == master_namespace and name in MASTER_SERVICES:
            out.setdefault(name, svc)
    return out


def from_services(services) -> list:
    """`envvars.FromServices`: in the given order, services without a cluster IP skipped; IPv6
    addresses are bracketed in the URL forms (`net.JoinHostPort`)."""
    env = []
    for svc in services:
        if not _ip_set(svc):
            continue
        name = _upper(svc["metadata"]["name"])
        spec = svc.get("spec") or {}
        ip = spec["clusterIP"]
        host = f"[{ip}]" if ":" in ip else ip
        ports = spec.get("ports") or []
        env.append({"name": f"{name}_SERVICE_HOST", "value": ip})
        if ports:
            env.append({"name": f"{name}_SERVICE_PORT", "value": str(ports[0]["port"])})
        for p in ports:
            if p.get("name"):
                env.append({"name": f"{name}_SERVICE_PORT_{_upper(p['name'])}", "value": str(p["port"])})
        for i, p in enumerate(ports):
            proto = (p.get("protocol") or "TCP").lower()
            url = f"{proto}://{host}:{p['port']}"
            prefix = f"{name}_PORT_{p['port']}_{proto.upper()}"
            if i == 0:
                env.append({"name": f"{name}_PORT", "value": url})
            env += [{"name": prefix, "value": url}, {"name": f"{prefix}_PROTO", "value": proto},
                    {"name": f"{prefix}_PORT", "value": str(p["port"])}, {"name": f"{prefix}_ADDR", "value": ip}]
    return env


def service_env(services, namespace, master_namespace=MASTER_NAMESPACE) -> list:
    return from_services(sorted(service_map(services, namespace, master_namespace).values(),
                                key=lambda s: s["metadata"]["name"]))
