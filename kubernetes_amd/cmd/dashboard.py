"""Cluster dashboard add-on (read-only web UI, GPU allocation first): addons/dashboard.py.

    python -m kubernetes_amd.cmd.dashboard --master http://127.0.0.1:8080 --port 9090
"""
from __future__ import annotations

import argparse
import os

from ..addons.dashboard import Dashboard
from ._common import run_until_signal, setup_logging


def main(argv=None):
    ap = argparse.ArgumentParser("dashboard")
    ap.add_argument("--master", default=os.environ.get("KUBERNETES_MASTER", "http://127.0.0.1:8080"))
    ap.add_argument("--token", default=None)
    ap.add_argument("--bind-address", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=9090)
    ap.add_argument("-v", type=int, default=0)
    a = ap.parse_args(argv)
    setup_logging(a.v)

    async def start():
        d = Dashboard(a.master, token=a.token)
        port = await d.start(a.bind_address, a.port)
        print(f"dashboard on :{port}", flush=True)
        return d

    run_until_signal(start)


if __name__ == "__main__":
    main()
