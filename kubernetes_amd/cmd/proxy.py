"""kube-proxy entry point (reference: cmd/kube-proxy/app/server.go:424, options :86-180)."""
from __future__ import annotations

import argparse
import os

from ..client.rest import Client
from ..proxy.server import ProxyServer
from ._common import run_until_signal, setup_logging


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
    ap.add_argument("-v", type=int, default=0)
    a = ap.parse_args(argv)
    setup_logging(a.v)
    if a.config:
        apply_config_file(a, a.config)

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
            client = client_from(a.kubeconfig)
        else:
            client = Client(a.master or "http://127.0.0.1:8080", token=a.token)
        ps = ProxyServer(client, a.hostname_override, a.proxy_mode, a.cluster_cidr,
                         a.masquerade_all, a.iptables_sync_period, a.iptables_min_sync_period,
                         healthz_port=a.healthz_port, metrics_port=a.metrics_port, iptables=iptables, ipvs=ipvs,
                         ipvs_scheduler=a.ipvs_scheduler, bind=a.bind_address)
        await ps.start()
        print(f"kube-proxy {a.hostname_override} running (mode={a.proxy_mode})", flush=True)
        return ps

    run_until_signal(start)


def _dur(v):
    from ..kubelet.kubeletconfig import parse_duration
    return parse_duration(v)


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
