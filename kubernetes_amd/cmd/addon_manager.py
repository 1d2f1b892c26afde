"""Add-on manager entry point (`cluster/addons/addon-manager`)."""
import argparse

from ..addons.manager import AddonManager
from ._common import run_until_signal, setup_logging


def main(argv=None):
    ap = argparse.ArgumentParser("kube-addon-manager")
    ap.add_argument("--kubeconfig", default=None)
    ap.add_argument("--master", default="http://127.0.0.1:8080")
    ap.add_argument("--addon-dir", default="/etc/kubernetes/addons")
    ap.add_argument("--period", type=float, default=60.0)
    ap.add_argument("-v", type=int, default=0)
    a = ap.parse_args(argv)
    setup_logging(a.v)

    async def start():
        import asyncio
        from ..client.clientcmd import client_from
        from ..client.rest import Client
        client = client_from(a.kubeconfig) if a.kubeconfig else Client(a.master)
        mgr = AddonManager(client, a.addon_dir, a.period)
        mgr.task = asyncio.ensure_future(mgr.run())
        return mgr

    run_until_signal(start)


if __name__ == "__main__":
    main()
