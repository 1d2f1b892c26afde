"""kamd-etcd-gateway: the etcd v3 gRPC API (KV, Watch, Lease, Maintenance.Status) in front of a
kamd-etcd store, for etcdctl and other etcd v3 clients (`storage/etcdv3.py`).

    python -m kubernetes_amd.cmd.etcd_gateway --store unix:///var/run/kamd-etcd.sock --listen 127.0.0.1:2379
    ETCDCTL_API=3 etcdctl --endpoints 127.0.0.1:2379 get /registry/ --prefix --keys-only
"""
from __future__ import annotations

import argparse

from ..storage.etcdv3 import EtcdV3Gateway
from ._common import run_until_signal, setup_logging


def main(argv=None):
    ap = argparse.ArgumentParser("kamd-etcd-gateway")
    ap.add_argument("--store", required=True, help="kamd-etcd address (unix:///path.sock or tcp://host:port)")
    ap.add_argument("--listen", default="127.0.0.1:2379")
    ap.add_argument("-v", type=int, default=0)
    a = ap.parse_args(argv)
    setup_logging(a.v)

    async def start():
        gw = await EtcdV3Gateway(a.store).start(a.listen)
        print(f"etcd v3 API for {a.store} on {a.listen.rsplit(':', 1)[0]}:{gw.port}", flush=True)
        return gw
    run_until_signal(start)


if __name__ == "__main__":
    main()
