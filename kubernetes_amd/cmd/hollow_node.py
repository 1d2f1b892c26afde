"""kubemark hollow-node entry point (reference: cmd/kubemark/hollow-node.go:46-160): N hollow
kubelets in one process, each with a fake 8 x MI355X amd.com/gpu plugin."""
from __future__ import annotations

import argparse

from ..kubemark.hollow import HollowCluster
from ._common import run_until_signal, setup_logging


def parse_links(spec):
    """'2-5,1-6' -> ((2, 5), (1, 6))"""
    return tuple(tuple(int(x) for x in p.split("-")) for p in spec.split(",") if p.strip())


def main(argv=None):
    ap = argparse.ArgumentParser("hollow-node")
    ap.add_argument("--master", required=True)
    ap.add_argument("--count", type=int, default=10)
    ap.add_argument("--name-prefix", default="hollow")
    ap.add_argument("--gpus-per-node", type=int, default=8)
    ap.add_argument("--hives", type=int, default=1)
    ap.add_argument("--partition", default="SPX", choices=["SPX", "DPX", "QPX", "CPX"],
                    help="compute-partition mode of the fake MI355X packages (CPX: 8 logical devices each)")
    ap.add_argument("--links-down", default="",
                    help="failed xGMI links of the fake packages, e.g. '2-5,1-6' (pairwise-topology fixtures)")
    ap.add_argument("--morph", default="kubelet", choices=["kubelet", "proxy"],
                    help="kubelet: hollow kubelets; proxy: hollow kube-proxies over a fake iptables (hollow-node.go:139+)")
    ap.add_argument("--payload-socket", default=None,
                    help="run each GPU container's payload through this PayloadServer (the rank holding the GPU)")
    ap.add_argument("--no-events", action="store_true")
    ap.add_argument("--node-status-update-frequency", type=float, default=10.0)
    ap.add_argument("--kube-api-content-type", default="application/vnd.kubernetes.protobuf",
                    choices=["application/json", "application/vnd.kubernetes.protobuf"],
                    help="the hollow kubelets' wire format (the kubelet's default: protobuf)")
    ap.add_argument("--ready-file", default=None, help="touched once every node's device plugin registered")
    ap.add_argument("-v", type=int, default=0)
    a = ap.parse_args(argv)
    setup_logging(a.v)

    async def start():
        if a.morph == "proxy":
            from ..client.rest import Client
            from ..proxy.iptables import FakeIptables
            from ..proxy.server import ProxyServer

            class Proxies:
                def __init__(self):
                    self.items = [ProxyServer(Client(a.master), f"{a.name_prefix}-{i}", "iptables", iptables=FakeIptables())
                                  for i in range(a.count)]

                async def stop(self):
                    for p in self.items:
                        await p.stop()
            ps = Proxies()
            for p in ps.items:
                await p.start()
            print(f"{a.count} hollow proxies syncing (fake iptables)", flush=True)
            return ps
        payload = None
        if a.payload_socket:
            from ..kubemark.payload import PayloadClient
            payload = PayloadClient(a.payload_socket)
        h = HollowCluster(a.master, a.count, a.name_prefix, a.gpus_per_node, a.hives, payload=payload,
                          emit_events=not a.no_events, status_freq=a.node_status_update_frequency,
                          partition=a.partition, links_down=parse_links(a.links_down),
                          content_type=a.kube_api_content_type)
        await h.start()
        await h.wait_registered()
        if a.ready_file:
            open(a.ready_file, "w").close()
        print(f"{a.count} hollow nodes registered ({a.gpus_per_node} GPUs each)", flush=True)
        return h

    run_until_signal(start)


if __name__ == "__main__":
    main()
