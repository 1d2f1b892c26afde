"""kube-proxy entry point (reference: cmd/kube-proxy/app/server.go:424, options :86-180)."""
from __future__ import annotations

import argparse
import os

from ..client.rest import Client
from ..proxy.server import ProxyServer
from ._common import check_unsupported, run_until_signal, setup_logging, unsupported


def main(argv=None):
    ap = argparse.ArgumentParser("kube-proxy")
    ap.add_argument("--master", default=None)
    ap.add_argument("--kubeconfig", default=None)
    ap.add_argument("--hostname-override", default=os.uname().nodename)
    ap.add_argument("--proxy-mode", default="iptables", choices=["iptables", "ipvs", "userspace"])
    ap.add_argument("--cluster-cidr", default="")
    ap.add_argument("--masquerade-all", action="store_true")
    ap.add_argument("--iptables-sync-period", type=float, default=30.0)
    ap.add_argument("--iptables-min-sync-period", type=float, default=0.0)
    ap.add_argument("--ipvs-scheduler", default="rr")
    ap.add_argument("--bind-address", default="127.0.0.1")
    ap.add_argument("--healthz-port", type=int, default=10256)
    ap.add_argument("--metrics-port", type=int, default=10249)
    ap.add_argument("--fake-dataplane", action="store_true",
                    help="record iptables/IPVS state without touching the kernel (kubemark hollow proxy)")
    ap.add_argument("--token", default=None)
    ap.add_argument("--config", default=None, help="KubeProxyConfiguration file (kubeproxy.config.k8s.io/v1alpha1)")
    _reference_flags(ap)
    ap.add_argument("-v", type=int, default=0)
    a = ap.parse_args(argv)
    check_unsupported(ap, a)
    setup_logging(a.v)
    if a.config:
        apply_config_file(a, a.config)
    for attr, port_attr in (("healthz_bind_address", "healthz_port"), ("metrics_bind_address", "metrics_port")):
        v = getattr(a, attr)
        if v and ":" in v:
            setattr(a, port_attr, int(v.rsplit(":", 1)[1]))
    if a.write_config_to:
        write_config(a, a.write_config_to)
        return
    if a.cleanup or a.cleanup_iptables or a.cleanup_ipvs:
        from ..proxy import cleanup as C
        ok = C.cleanup_iptables() if (a.cleanup or a.cleanup_iptables) else True
        if a.cleanup or a.cleanup_ipvs:
            ok = C.cleanup_ipvs() and ok
        raise SystemExit(0 if ok else 1)
    if a.proxy_mode == "ipvs":
        a.iptables_sync_period = _dur(a.ipvs_sync_period)
        a.iptables_min_sync_period = _dur(a.ipvs_min_sync_period)
    if not a.fake_dataplane:
        from ..kubelet.hostchecks import set_oom_score_adj
        from ..proxy.cleanup import conntrack_max, set_conntrack
        set_oom_score_adj(a.oom_score_adj)
        set_conntrack(conntrack_max(a.conntrack_max_per_core, a.conntrack_min) or a.conntrack_max,
                      int(_dur(a.conntrack_tcp_timeout_established)))

    async def start():
        iptables = ipvs = None
        if not a.fake_dataplane:
            if a.proxy_mode == "iptables":
                from ..proxy.iptables import ExecIptables
                iptables = ExecIptables()
            elif a.proxy_mode == "ipvs":
                from ..proxy.ipvs import ExecIPVS
                ipvs = ExecIPVS()
        if a.kubeconfig:
            from ..client.clientcmd import client_from
            client = client_from(a.kubeconfig, qps=a.kube_api_qps, burst=a.kube_api_burst, content_type=a.kube_api_content_type)
        else:
            client = Client(a.master or "http://127.0.0.1:8080", token=a.token, qps=a.kube_api_qps, burst=a.kube_api_burst,
                            content_type=a.kube_api_content_type)
        ps = ProxyServer(client, a.hostname_override, a.proxy_mode, a.cluster_cidr,
                         a.masquerade_all, a.iptables_sync_period, a.iptables_min_sync_period,
                         healthz_port=a.healthz_port, metrics_port=a.metrics_port, iptables=iptables, ipvs=ipvs,
                         ipvs_scheduler=a.ipvs_scheduler, bind=a.bind_address, masquerade_bit=a.iptables_masquerade_bit,
                         resync=_dur(a.config_sync_period), profiling=a.profiling)
        await ps.start()
        print(f"kube-proxy {a.hostname_override} running (mode={a.proxy_mode})", flush=True)
        return ps

    run_until_signal(start)


def _dur(v):
    from ..kubelet.kubeletconfig import parse_duration
    if isinstance(v, (int, float)):
        return float(v)
    return parse_duration(v)


def _bool(v):
    return str(v).lower() not in ("false", "0", "no")


def _reference_flags(ap):
    """The rest of kube-proxy's flags (cmd/kube-proxy/app/server.go AddFlags)."""
    ap.add_argument("--cleanup", action="store_true", help="remove iptables and IPVS rules kube-proxy made, then exit")
    ap.add_argument("--cleanup-iptables", action="store_true", help="deprecated: remove the iptables rules, then exit")
    ap.add_argument("--cleanup-ipvs", type=_bool, default=False, help="remove the IPVS rules, then exit")
    ap.add_argument("--write-config-to", default="", help="write the effective KubeProxyConfiguration here and exit")
    ap.add_argument("--healthz-bind-address", default="", help="ip:port (overrides --healthz-port)")
    ap.add_argument("--metrics-bind-address", default="", help="ip:port (overrides --metrics-port)")
    ap.add_argument("--iptables-masquerade-bit", type=int, default=14)
    ap.add_argument("--ipvs-sync-period", default="30s")
    ap.add_argument("--ipvs-min-sync-period", default="0s")
    ap.add_argument("--conntrack-max", type=int, default=0, help="deprecated absolute limit (0 = use per-core)")
    ap.add_argument("--conntrack-max-per-core", type=int, default=32768)
    ap.add_argument("--conntrack-min", type=int, default=131072)
    ap.add_argument("--conntrack-tcp-timeout-established", default="24h")
    ap.add_argument("--oom-score-adj", type=int, default=-999)
    ap.add_argument("--kube-api-qps", type=float, default=5.0)
    ap.add_argument("--kube-api-burst", type=int, default=10)
    ap.add_argument("--kube-api-content-type", default="application/vnd.kubernetes.protobuf",
                    choices=["application/json", "application/vnd.kubernetes.protobuf"],
                    help="wire format of API requests and watch streams (reference default protobuf, "
                         "`pkg/apis/componentconfig/v1alpha1/defaults.go:75`: protobuf bodies and "
                         "length-delimited protobuf watch frames, decoded natively)")
    ap.add_argument("--config-sync-period", default="15m",
                    help="the service/endpoints informers re-deliver every object every [p, 2p), re-syncing the rules")
    unsupported(ap, "--proxy-port-range", "", str, "userspace-mode proxy ports come from the OS")
    unsupported(ap, "--udp-timeout", "250ms", str, "the userspace proxier keeps no UDP sessions")
    unsupported(ap, "--resource-container", "", str, "kube-proxy is not moved into a cgroup of its own")
    ap.add_argument("--profiling", type=_bool, default=False, help="serve /debug/pprof on the metrics port")


def write_config(a, path):
    import yaml
    cfg = {"apiVersion": "kubeproxy.config.k8s.io/v1alpha1", "kind": "KubeProxyConfiguration",
           "bindAddress": a.bind_address, "clusterCIDR": a.cluster_cidr, "hostnameOverride": a.hostname_override,
           "mode": a.proxy_mode, "healthzBindAddress": f"{a.bind_address}:{a.healthz_port}",
           "metricsBindAddress": f"{a.bind_address}:{a.metrics_port}", "oomScoreAdj": a.oom_score_adj,
           "clientConnection": {"kubeconfig": a.kubeconfig or "", "qps": a.kube_api_qps, "burst": a.kube_api_burst},
           "iptables": {"masqueradeAll": a.masquerade_all, "masqueradeBit": a.iptables_masquerade_bit,
                        "syncPeriod": f"{a.iptables_sync_period}s", "minSyncPeriod": f"{a.iptables_min_sync_period}s"},
           "ipvs": {"scheduler": a.ipvs_scheduler, "syncPeriod": a.ipvs_sync_period, "minSyncPeriod": a.ipvs_min_sync_period},
           "conntrack": {"max": a.conntrack_max, "maxPerCore": a.conntrack_max_per_core, "min": a.conntrack_min,
                         "tcpEstablishedTimeout": a.conntrack_tcp_timeout_established}}
    with open(path, "w") as f:
        yaml.safe_dump(cfg, f, sort_keys=False)


def apply_config_file(a, path):
    """`pkg/proxy/apis/kubeproxyconfig` KubeProxyConfiguration → flag values (the file wins,
    as `--config` does in the reference)."""
    import yaml
    with open(path) as f:
        c = yaml.safe_load(f) or {}
    if c.get("kind", "KubeProxyConfiguration") != "KubeProxyConfiguration":
        raise SystemExit(f"kube-proxy: {path}: expected kind KubeProxyConfiguration")
    a.proxy_mode = c.get("mode") or a.proxy_mode
    a.cluster_cidr = c.get("clusterCIDR", a.cluster_cidr)
    a.bind_address = c.get("bindAddress", a.bind_address)
    a.hostname_override = c.get("hostnameOverride") or a.hostname_override
    ipt = c.get("iptables") or {}
    a.masquerade_all = ipt.get("masqueradeAll", a.masquerade_all)
    if "syncPeriod" in ipt:
        a.iptables_sync_period = _dur(ipt["syncPeriod"])
    if "minSyncPeriod" in ipt:
        a.iptables_min_sync_period = _dur(ipt["minSyncPeriod"])
    ipvs = c.get("ipvs") or {}
    a.ipvs_scheduler = ipvs.get("scheduler") or a.ipvs_scheduler
    for key, attr in (("healthzBindAddress", "healthz_port"), ("metricsBindAddress", "metrics_port")):
        v = c.get(key)
        if v and ":" in str(v):
            setattr(a, attr, int(str(v).rsplit(":", 1)[1]))
    kc = (c.get("clientConnection") or {}).get("kubeconfig")
    if kc:
        a.kubeconfig = kc
    return a


if __name__ == "__main__":
    main()
