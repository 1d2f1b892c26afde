"""kube-apiserver entry point (reference: cmd/kube-apiserver/app/server.go:102-132)."""
from __future__ import annotations

import argparse

from ..api import codec
from ..apiserver.server import APIServer
from ..storage.mvcc import MVCCStore
from ._common import run_until_signal, setup_logging, write_port_file


def main(argv=None):
    ap = argparse.ArgumentParser("kube-apiserver")
    ap.add_argument("--bind-address", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=8080)
    ap.add_argument("--port-file", default=None, help="write the bound port here (use with --port 0)")
    ap.add_argument("--admission-control", default=None, help="comma separated ordered plugin list")
    ap.add_argument("--authorization-mode", default="AlwaysAllow")
    ap.add_argument("--token-auth-file", default=None)
    ap.add_argument("--storage-media-type", default=codec.JSON)
    ap.add_argument("--storage-engine", default="native", choices=["native", "python"])
    ap.add_argument("--etcd-wal", default=None, help="durable WAL path for the embedded store")
    ap.add_argument("--max-requests-inflight", type=int, default=4000)
    ap.add_argument("--max-mutating-requests-inflight", type=int, default=2000)
    ap.add_argument("--watch-cache-size", type=int, default=200000)
    ap.add_argument("-v", type=int, default=0)
    a = ap.parse_args(argv)
    setup_logging(a.v)

    async def start():
        store = None
        if a.storage_engine == "native":
            try:
                from ..storage.native_store import NativeMVCCStore
                store = NativeMVCCStore(wal_path=a.etcd_wal)
            except (ImportError, OSError):
                store = None
        if store is None:
            store = MVCCStore(wal_path=a.etcd_wal)
        plugins = a.admission_control.split(",") if a.admission_control else None
        s = APIServer(store=store, admission_plugins=plugins, token_file=a.token_auth_file,
                      authorization_modes=a.authorization_mode.split(","), storage_media_type=a.storage_media_type,
                      max_requests_inflight=a.max_requests_inflight,
                      max_mutating_inflight=a.max_mutating_requests_inflight, watch_window=a.watch_cache_size)
        port = await s.start(a.bind_address, a.port)
        write_port_file(a.port_file, port)
        print(f"kube-apiserver listening on http://{a.bind_address}:{port}", flush=True)
        return s

    run_until_signal(start)


if __name__ == "__main__":
    main()
