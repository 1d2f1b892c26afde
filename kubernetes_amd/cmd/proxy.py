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
    ap.add_argument("-v", type=int, default=0)
    a = ap.parse_args(argv)
    setup_logging(a.v)

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


if __name__ == "__main__":
    main()
