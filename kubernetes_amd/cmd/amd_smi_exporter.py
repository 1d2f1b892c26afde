"""Standalone amd-smi Prometheus exporter (:9400)."""
from __future__ import annotations

import argparse

from ..monitoring.exporter import AMDSMIExporter, kubelet_pods_fn, kubelet_stats_fn
from ..native import amdsmi
from ._common import run_until_signal, setup_logging


def main(argv=None):
    ap = argparse.ArgumentParser("amd-smi-exporter")
    ap.add_argument("--port", type=int, default=9400)
    ap.add_argument("--node-name", default="")
    ap.add_argument("--kubelet", default=None, help="kubelet URL for pod attribution, e.g. http://127.0.0.1:10250")
    ap.add_argument("--fixture", default=None)
    ap.add_argument("-v", type=int, default=0)
    a = ap.parse_args(argv)
    setup_logging(a.v)

    async def start():
        ex = AMDSMIExporter(amdsmi.SMI(fixture=a.fixture), a.node_name,
                            pods_fn=kubelet_pods_fn(a.kubelet) if a.kubelet else None,
                            stats_fn=kubelet_stats_fn(a.kubelet) if a.kubelet else None)
        port = await ex.start("0.0.0.0", a.port)
        print(f"amd-smi exporter serving {len(ex.gpus)} GPU(s) on :{port}", flush=True)
        return ex

    run_until_signal(start)


if __name__ == "__main__":
    main()
