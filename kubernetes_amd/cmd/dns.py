"""Cluster DNS server entry point (kube-dns equivalent)."""
import argparse
import os

from ..addons.dns import DNSServer
from ._common import run_until_signal, setup_logging, write_port_file


def main(argv=None):
    ap = argparse.ArgumentParser("kube-dns")
    ap.add_argument("--kubeconfig", default=None)
    ap.add_argument("--master", default=None)
    ap.add_argument("--domain", default="cluster.local")
    ap.add_argument("--bind-address", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=53)
    ap.add_argument("--port-file", default=None)
    ap.add_argument("--upstream", action="append", default=[], help="upstream resolver host[:port] (default: resolv.conf)")
    ap.add_argument("-v", type=int, default=0)
    a = ap.parse_args(argv)
    setup_logging(a.v)

    async def start():
        from ..client.clientcmd import client_from
        from ..client.rest import Client
        from ..kubelet.network import parse_resolv_conf
        client = client_from(a.kubeconfig) if a.kubeconfig else Client(a.master or os.environ.get(
            "KUBERNETES_MASTER", "http://127.0.0.1:8080"))
        ups = a.upstream or parse_resolv_conf("/etc/resolv.conf")[0]
        srv = DNSServer(client, a.domain, ups)
        port = await srv.start(a.bind_address, a.port)
        write_port_file(a.port_file, port)
        print(f"kube-dns serving {a.domain} on {a.bind_address}:{port} (udp+tcp), upstreams {ups}", flush=True)
        return srv

    run_until_signal(start)


if __name__ == "__main__":
    main()
