"""Host-path CSI driver (+ optional external-attacher sidecar) entry point."""
import argparse
import os

from ._common import run_until_signal, setup_logging


def main(argv=None):
    ap = argparse.ArgumentParser("csi-hostpath")
    ap.add_argument("--drivername", default="hostpath.csi.amd.com")
    ap.add_argument("--endpoint", default="/var/lib/kubelet/plugins/hostpath.csi.amd.com/csi.sock")
    ap.add_argument("--nodeid", default=os.uname().nodename)
    ap.add_argument("--data-dir", default="/var/lib/csi-hostpath")
    ap.add_argument("--attacher", action="store_true", help="also run the external attacher against the API")
    ap.add_argument("--kubeconfig", default=None)
    ap.add_argument("--master", default="http://127.0.0.1:8080")
    ap.add_argument("-v", type=int, default=0)
    a = ap.parse_args(argv)
    setup_logging(a.v)

    async def start():
        from ..csi.driver import HostPathDriver
        drv = await HostPathDriver(a.drivername, a.data_dir, a.nodeid).start(a.endpoint)
        print(f"csi-hostpath {a.drivername} serving on unix://{a.endpoint}", flush=True)
        if a.attacher:
            from ..client.clientcmd import client_from
            from ..client.rest import Client
            from ..controllers.manager import ControllerManager
            client = client_from(a.kubeconfig) if a.kubeconfig else Client(a.master)
            cm = ControllerManager(client, ["csi-attacher"], {"csi-attacher": {"driver": a.drivername,
                                                                              "endpoint": a.endpoint}})
            await cm.start()
        return drv

    run_until_signal(start)


if __name__ == "__main__":
    main()
